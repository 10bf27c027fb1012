#!/bin/bash
# GPU box: single-GPU decode + first-token bench of the other BASELINE models
set -o pipefail
mkdir -p gpurun_out
for m in llama3-70b mixtral-8x7b; do for b in 1 8; do
  timeout -k 10 400 python bench.py --model $m --batch $b --steps 32 --warmup 4 > gpurun_out/bench_${m}_b$b.log 2>&1 || exit $?
  echo "$m B=$b $(tail -1 gpurun_out/bench_${m}_b$b.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"first_token_latency_ms": [0-9.]*' | tr '\n' ' ')"
done; done
