#!/bin/bash
# re-entry check: streaming-chain probe, then B=1 / B=8 headline bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 240 tools/probe/layer_probe > gpurun_out/layer_probe.jsonl 2>&1 || exit $?
for b in 1 8; do
  BENCH_BATCH=$b timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench_b$b.log 2>&1 || exit $?
  tail -1 gpurun_out/bench_b$b.log | cut -c1-250
done
