#!/bin/bash
# deferred-norm + GEMV geometry: probe timings, kernel/model GPU tests, B=1/4/8 bench
set -o pipefail
mkdir -p gpurun_out
PROBE_MODE=d timeout -k 10 200 tools/probe/gemv5_probe_w1 > gpurun_out/gemv5_defer.jsonl 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pt_r3n.log 2>&1
rc=$?; tail -5 gpurun_out/pt_r3n.log; [ $rc -ne 0 ] && exit $rc
for b in 1 4 8; do
  BENCH_BATCH=$b timeout -k 10 300 python bench.py --steps 32 --warmup 4 > gpurun_out/bench_b$b.log 2>&1 || exit $?
  tail -1 gpurun_out/bench_b$b.log | cut -c1-200
done
for b in 1 8; do
  ILLM_DEFER_NORM=0 BENCH_BATCH=$b timeout -k 10 300 python bench.py --steps 32 --warmup 4 > gpurun_out/bench_nodefer_b$b.log 2>&1 || exit $?
  tail -1 gpurun_out/bench_nodefer_b$b.log | cut -c1-200
done
