#!/bin/bash
# round 5: attention -> o_proj chained launch: tests, then decode A/B (ILLM_ATTN_OPROJ=0/1) at B = 8 / 1
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread -k "oproj_chain" > gpurun_out/r5z_pytest.log 2>&1 || { tail -40 gpurun_out/r5z_pytest.log; exit 2; }
grep -c PASSED gpurun_out/r5z_pytest.log
: > gpurun_out/r5z_ab.jsonl
run() {  # B, flag
  ILLM_ATTN_OPROJ=$2 BENCH_BATCH=$1 timeout -k 10 200 python bench.py --steps 64 --warmup 8 --no-tp-side > gpurun_out/r5z_tmp.log 2>&1 || { tail -5 gpurun_out/r5z_tmp.log; return 1; }
  tail -1 gpurun_out/r5z_tmp.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(json.dumps({'B': $1, 'attn_oproj': $2, 'tok_s': d['value'], 'ms': d['ms_per_step']}))" | tee -a gpurun_out/r5z_ab.jsonl
}
for i in 1 2; do
  for fl in 1 0; do run 8 $fl || exit 3; done
  for fl in 1 0; do run 1 $fl || exit 3; done
done
