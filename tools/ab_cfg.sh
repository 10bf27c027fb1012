#!/bin/bash
# A/B of environment configurations on the decode bench (GPU box).
# usage: bash tools/ab_cfg.sh "B1 B2" "label1:VAR=v,VAR2=v" "label2:..." ...
# Each config runs bench.py once per batch size; prints ms/step per config.
set -o pipefail
mkdir -p gpurun_out
BS=$1; shift
for b in $BS; do
  for cfg in "$@"; do
    label=${cfg%%:*}; envs=${cfg#*:}
    envargs=$(echo "$envs" | tr ',' ' ')
    env $envargs BENCH_BATCH=$b timeout -k 10 300 python bench.py --steps 64 --warmup 8 > gpurun_out/abc_${label}_b$b.log 2>&1 || { tail -20 gpurun_out/abc_${label}_b$b.log; exit 1; }
    echo "$label B=$b $(tail -1 gpurun_out/abc_${label}_b$b.log | grep -o '"ms_per_step": [0-9.]*') $(tail -1 gpurun_out/abc_${label}_b$b.log | grep -o '"sample_next_ids": \[[0-9, ]*')"
  done
done
