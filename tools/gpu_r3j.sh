#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_bounds.py tests/test_gpu_dense_gemv.py tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_families.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pt_r3j.log 2>&1
rc=$?
tail -3 gpurun_out/pt_r3j.log
[ $rc -ne 0 ] && exit $rc
for b in 1 8; do
  BENCH_BATCH=$b timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench_b$b.log 2>&1 || exit $?
  tail -1 gpurun_out/bench_b$b.log | cut -c1-250
done
