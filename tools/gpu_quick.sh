#!/bin/bash
# GPU-box pass: gpu tests (stop at first failure), GEMV micro-bench, B=1/B=8 decode bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -15 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/bench_kernels.py --only gemv > gpurun_out/bk_gemv.log 2>&1 || exit $?
BENCH_BATCH=1 timeout -k 10 300 python bench.py --steps 64 --warmup 8 > gpurun_out/bench_b1.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 64 --warmup 8 > gpurun_out/bench_b8.log 2>&1 || exit $?
cat gpurun_out/bk_gemv.log | cut -c1-150
tail -1 gpurun_out/bench_b1.log | cut -c1-300; tail -1 gpurun_out/bench_b8.log | cut -c1-300
