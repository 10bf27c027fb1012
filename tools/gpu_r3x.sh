#!/bin/bash
# other BASELINE models + long context + TP/EP flags at world 1 with the round-3 decode path
set -o pipefail
mkdir -p gpurun_out
for m in llama3-70b mixtral-8x7b; do for b in 1 8; do
  timeout -k 10 400 python bench.py --model $m --batch $b --steps 32 --warmup 4 > gpurun_out/bench_${m}_b$b.log 2>&1 || exit $?
  echo "$m B=$b $(tail -1 gpurun_out/bench_${m}_b$b.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"first_token_latency_ms": [0-9.]*' | tr '\n' ' ')"
done; done
timeout -k 10 400 python bench.py --model llama3-70b --tp --batch 8 --steps 16 --warmup 2 > gpurun_out/bench_70b_tp1.log 2>&1 || exit $?
echo "70b --tp (world 1) $(tail -1 gpurun_out/bench_70b_tp1.log | grep -o '"ms_per_step": [0-9.]*\|"parallelism": "[a-z0-9]*"' | tr '\n' ' ')"
timeout -k 10 400 python bench.py --model mixtral-8x7b --ep --batch 8 --steps 16 --warmup 2 > gpurun_out/bench_mix_ep1.log 2>&1 || exit $?
echo "mixtral --ep (world 1) $(tail -1 gpurun_out/bench_mix_ep1.log | grep -o '"ms_per_step": [0-9.]*\|"parallelism": "[a-z0-9]*"' | tr '\n' ' ')"
for p in 8192 32768; do
  BENCH_BATCH=1 timeout -k 10 400 python bench.py --prompt-len $p --steps 32 --warmup 4 > gpurun_out/bench_b1_p$p.log 2>&1 || exit $?
  echo "B=1 prompt $p $(tail -1 gpurun_out/bench_b1_p$p.log | grep -o '"ms_per_step": [0-9.]*\|"first_token_latency_ms": [0-9.]*' | tr '\n' ' ')"
done
