#!/bin/bash
# A/B of one environment switch on the B=1 and B=8 decode bench (GPU box).
# usage: bash tools/ab_env.sh VAR "valA valB" [pytest -k expr]
set -o pipefail
mkdir -p gpurun_out
VAR=$1; VALS=$2; K=$3
if [ -n "$K" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$K" > gpurun_out/pytest_ab.log 2>&1 || { tail -30 gpurun_out/pytest_ab.log; exit 1; }
  tail -2 gpurun_out/pytest_ab.log
fi
for b in 1 8; do
  for v in $VALS; do
    env $VAR=$v BENCH_BATCH=$b timeout -k 10 300 python bench.py --steps 64 --warmup 8 > gpurun_out/ab_${VAR}_${v}_b$b.log 2>&1 || exit $?
    echo "$VAR=$v B=$b $(tail -1 gpurun_out/ab_${VAR}_${v}_b$b.log | grep -o '"ms_per_step": [0-9.]*') $(tail -1 gpurun_out/ab_${VAR}_${v}_b$b.log | grep -o '"first_token_latency_ms": [0-9.]*')"
  done
done
