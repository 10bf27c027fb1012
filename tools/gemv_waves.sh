#!/bin/bash
set -e
mkdir -p gpurun_out
for w in 4 8; do
  ILLM_GEMV_WAVES=$w timeout -k 10 200 python tools/bench_kernels.py --m 1,4,8,16 --only gemv > gpurun_out/waves_$w.log 2>&1
done
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_moe.py -x -q > gpurun_out/pytest_k.log 2>&1
