#!/bin/bash
# round 5: full GPU suite + 8-phase low-bit decode-schedule sweep (ILLM_G8_SCHED 0/1/2)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
for s in 0 1 2; do
  ILLM_G8_SCHED=$s timeout -k 10 240 python -u tools/bench_g8.py sym_int4 --m 8192,1024 $([ $s = 0 ] && echo --dense) > gpurun_out/r5f_g8_s$s.jsonl 2> gpurun_out/r5f_g8_s$s.err || exit 3
  echo "sched $s done"
done
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 280 --timeout-method thread > gpurun_out/r5f_pytest.log 2>&1
rc=$?
tail -8 gpurun_out/r5f_pytest.log
exit $rc
