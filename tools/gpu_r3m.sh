#!/bin/bash
# GEMV geometry x occupancy sweep (production v5 kernel in a standalone probe)
set -o pipefail
mkdir -p gpurun_out
for w in 1 2 4; do
  timeout -k 10 200 tools/probe/gemv5_probe_w$w >> gpurun_out/gemv5_sweep.jsonl 2>&1 || exit $?
done
