#!/bin/bash
# prefill GEMM auto block shape: numerics + first-token A/B (ILLM_GEMM_TILE=0 = previous 128x128 everywhere)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_moe_gemm.py tests/test_gpu_moe.py -x -q --timeout 200 --timeout-method thread -k "gemm or moe" > gpurun_out/pt_r3ad.log 2>&1
rc=$?; tail -2 gpurun_out/pt_r3ad.log; [ $rc -ne 0 ] && exit $rc
for cfg in "1 auto" "1 0" "8 auto" "8 0"; do
  set -- $cfg
  if [ $2 = auto ]; then e=""; else e="ILLM_GEMM_TILE=$2"; fi
  env $e BENCH_BATCH=$1 timeout -k 10 300 python bench.py --steps 16 --warmup 2 > gpurun_out/ttft_t$2_b$1.log 2>&1 || exit $?
  echo "b=$1 tile=$2 $(tail -1 gpurun_out/ttft_t$2_b$1.log | grep -o '"first_token_latency_ms": [0-9.]*')"
done
for t in auto 0; do
  if [ $t = auto ]; then e=""; else e="ILLM_GEMM_TILE=$t"; fi
  env $e BENCH_BATCH=1 timeout -k 10 400 python bench.py --model mixtral-8x7b --steps 8 --warmup 2 > gpurun_out/ttft_mix_t$t.log 2>&1 || exit $?
  echo "mixtral b=1 tile=$t $(tail -1 gpurun_out/ttft_mix_t$t.log | grep -o '"first_token_latency_ms": [0-9.]*')"
done
