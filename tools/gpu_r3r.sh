#!/bin/bash
# GEMV-epilogue RoPE tests + A/B bench; shared-scale-window GEMV probe A/B
set -o pipefail
mkdir -p gpurun_out
for v in s0 s1 s1p4; do
  PROBE_MODE=d timeout -k 10 200 tools/probe/gemv5_probe_$v > gpurun_out/gemv5_scl_$v.jsonl 2>&1 || exit $?
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pt_r3q.log 2>&1
rc=$?; tail -5 gpurun_out/pt_r3q.log; [ $rc -ne 0 ] && exit $rc
for b in 1 8 4; do
  for r in 1 0; do
    ILLM_GEMV_ROPE=$r BENCH_BATCH=$b timeout -k 10 300 python bench.py --steps 64 --warmup 4 > gpurun_out/ab_rope${r}_b$b.log 2>&1 || exit $?
    echo "b=$b rope=$r $(tail -1 gpurun_out/ab_rope${r}_b$b.log | grep -o '"ms_per_step": [0-9.]*')"
  done
done
