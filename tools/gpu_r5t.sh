#!/bin/bash
# round 5: batched-row norm-in prologue (GLU norm-in at batch 8 vs standalone norm + GLU)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "norm_in or decode" > gpurun_out/r5t_pytest.log 2>&1 || { tail -30 gpurun_out/r5t_pytest.log; exit 2; }
tail -2 gpurun_out/r5t_pytest.log
: > gpurun_out/r5t_ab.jsonl
for i in 1 2; do
  for v in 4 8; do
    ILLM_DEFER_GLU_MAX_M=$v BENCH_BATCH=8 timeout -k 10 200 python bench.py --steps 64 --warmup 8 --no-tp-side > gpurun_out/r5t_tmp.log 2>&1 || { tail -5 gpurun_out/r5t_tmp.log; exit 3; }
    tail -1 gpurun_out/r5t_tmp.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(json.dumps({'B': 8, 'defer_glu_max_m': $v, 'tok_s': d['value'], 'ms': d['ms_per_step']}))" | tee -a gpurun_out/r5t_ab.jsonl
  done
done
