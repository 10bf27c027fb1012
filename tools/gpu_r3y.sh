#!/bin/bash
# attention combine merged into the o_proj GEMV prologue (with deferred norm + GEMV RoPE): A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread -k "attn or oproj or split or deferred" > gpurun_out/pt_r3y.log 2>&1
rc=$?; tail -2 gpurun_out/pt_r3y.log; [ $rc -ne 0 ] && exit $rc
for b in 1 4; do
  for cfg in "0 32" "1 32" "1 8" "0 32"; do
    set -- $cfg
    ILLM_OPROJ_COMBINE=$1 ILLM_OPROJ_KS=$2 BENCH_BATCH=$b timeout -k 10 300 python bench.py --steps 64 --warmup 4 > gpurun_out/ab_oc$1_ks$2_b$b.log 2>&1 || exit $?
    echo "b=$b oproj_combine=$1 ks=$2 $(tail -1 gpurun_out/ab_oc$1_ks$2_b$b.log | grep -o '"ms_per_step": [0-9.]*')"
  done
done
