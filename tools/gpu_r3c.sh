#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kquant.py tests/test_gpu_allreduce.py tests/test_gpu_tp.py tests/test_gpu_moe_gemm.py tests/test_gpu_moe.py -x -v --timeout 200 --timeout-method thread > gpurun_out/pt_r3c.log 2>&1
rc=$?
tail -4 gpurun_out/pt_r3c.log
[ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ] && exit $rc
BENCH_BATCH=1 timeout -k 10 300 python bench.py --model mixtral-8x7b --steps 32 --warmup 4 > gpurun_out/mixtral_b1.log 2>&1 || exit $?
tail -1 gpurun_out/mixtral_b1.log | cut -c1-600
BENCH_BATCH=8 timeout -k 10 300 python bench.py --model mixtral-8x7b --steps 32 --warmup 4 > gpurun_out/mixtral_b8.log 2>&1 || exit $?
tail -1 gpurun_out/mixtral_b8.log | cut -c1-600
