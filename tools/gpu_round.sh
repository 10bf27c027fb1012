#!/bin/bash
# One GPU-box pass: gpu tests, B=1/B=8 bench, rocprofv3 kernel stats of the decode bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
cd "$R"
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
BENCH_BATCH=1 timeout -k 10 300 python bench.py --steps 64 --warmup 8 > gpurun_out/bench_b1.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 64 --warmup 8 > gpurun_out/bench_b8.log 2>&1 || exit $?
tail -1 gpurun_out/bench_b1.log | cut -c1-400; tail -1 gpurun_out/bench_b8.log | cut -c1-400
bash tools/prof_decode.sh || exit $?
exit $rc
