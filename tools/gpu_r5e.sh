#!/bin/bash
# round 5: full GPU suite, bench A/B (argmax epilogue), decode traces, o / lm_head geometry sweep
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 280 --timeout-method thread > gpurun_out/r5e_pytest.log 2>&1
rc=$?
tail -5 gpurun_out/r5e_pytest.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
for B in 8 1; do
  for e in 1 0; do
    ILLM_ARGMAX_EPI=$e BENCH_BATCH=$B timeout -k 10 200 python bench.py --steps 64 --warmup 8 > gpurun_out/r5e_bench_b${B}_a$e.log 2>&1 || exit 3
    echo "B=$B argmax_epi=$e: $(tail -1 gpurun_out/r5e_bench_b${B}_a$e.log | cut -c1-330)"
  done
done
bash tools/prof_decode.sh || exit $?
head -16 gpurun_out/prof_b1_summary.txt; head -18 gpurun_out/prof_b8_summary.txt
bash tools/gpu_r5d.sh || exit 4
exit $rc
