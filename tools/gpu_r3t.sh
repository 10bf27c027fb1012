#!/bin/bash
# GLU shared-scale window + vectorised fused-combine hand-off: GPU tests, bench A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_moe.py tests/test_gpu_moe_gemm.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pt_r3t.log 2>&1
rc=$?; tail -3 gpurun_out/pt_r3t.log; [ $rc -ne 0 ] && exit $rc
for b in 1 8; do
  for fc in 0 1 0 1; do
    ILLM_ATTN_FUSED_COMBINE=$fc BENCH_BATCH=$b timeout -k 10 300 python bench.py --steps 64 --warmup 4 > gpurun_out/ab_fc${fc}_b$b.log 2>&1 || exit $?
    echo "b=$b fc=$fc $(tail -1 gpurun_out/ab_fc${fc}_b$b.log | grep -o '"ms_per_step": [0-9.]*')"
  done
done
