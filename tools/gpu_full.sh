#!/bin/bash
# GPU box: full gpu test suite + smoke() + headline bench (B=1 / B=8)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -4 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
BENCH_BATCH=1 timeout -k 10 300 python bench.py --steps 64 --warmup 8 > gpurun_out/bench_b1.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 64 --warmup 8 > gpurun_out/bench_b8.log 2>&1 || exit $?
tail -1 gpurun_out/bench_b1.log | cut -c1-330; tail -1 gpurun_out/bench_b8.log | cut -c1-330
exit $rc
