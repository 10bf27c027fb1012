#!/bin/bash
# GEMV prefetch-depth / split-K sweep + per-kernel floor (GPU box)
set -e
mkdir -p gpurun_out
timeout -k 10 300 python tools/bench_kernels.py --m 1,8 --ks 0,2,4,8,16 > gpurun_out/sweep_pf4.log 2>&1
ILLM_GEMV_PF=8 timeout -k 10 300 python tools/bench_kernels.py --m 1,8 --only gemv > gpurun_out/sweep_pf8.log 2>&1
ILLM_GEMV_PF=16 timeout -k 10 300 python tools/bench_kernels.py --m 1,8 --only gemv > gpurun_out/sweep_pf16.log 2>&1
