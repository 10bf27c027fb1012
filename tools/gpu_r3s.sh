#!/bin/bash
# shared-scale-window GEMV probe A/B; resident dense prefill shadow TTFT A/B
set -o pipefail
mkdir -p gpurun_out
for v in s0 s1 s1p4; do
  PROBE_MODE=d timeout -k 10 200 tools/probe/gemv5_probe_$v > gpurun_out/gemv5_scl2_$v.jsonl 2>&1 || exit $?
done
for b in 1 8; do
  for gb in 0 40; do
    ILLM_PREFILL_DENSE_GB=$gb BENCH_BATCH=$b timeout -k 10 300 python bench.py --steps 16 --warmup 2 > gpurun_out/ttft_gb${gb}_b$b.log 2>&1 || exit $?
    echo "b=$b gb=$gb $(tail -1 gpurun_out/ttft_gb${gb}_b$b.log | grep -o '"first_token_latency_ms": [0-9.]*')"
  done
done
