#!/bin/bash
# round 5: GEMV x staging by LDS-DMA (batch-8 gate/up): tests, GLU sweep, bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5y_pytest.log 2>&1 || { tail -30 gpurun_out/r5y_pytest.log; exit 2; }
tail -2 gpurun_out/r5y_pytest.log
timeout -k 10 200 python tools/gemv_sweep5.py 1,4,8,16 glu > gpurun_out/r5y_glu.jsonl || exit 3
cat gpurun_out/r5y_glu.jsonl
for B in 8 8 1; do
  BENCH_BATCH=$B timeout -k 10 200 python bench.py --steps 64 --warmup 8 --no-tp-side > gpurun_out/r5y_b$B.log 2>&1 || { tail -5 gpurun_out/r5y_b$B.log; exit 4; }
  echo "B=$B $(tail -1 gpurun_out/r5y_b$B.log | grep -o '"ms_per_step": [0-9.]*')"
done
