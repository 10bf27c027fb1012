#!/bin/bash
# round 5: one call for the pending measurements: v3 NW re-sweep, full-K store GEMV sweep, norm-in A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
bash tools/gpu_r5t.sh || exit $?
: > gpurun_out/r5r_attn.jsonl
for nw in 2 8; do
  for B in 1 8; do
    ILLM_ATTN_V3_NW=$nw timeout -k 10 120 python tools/bench_attn_dec.py $B 1025 20 >> gpurun_out/r5r_attn.jsonl || exit 4
  done
done
cat gpurun_out/r5r_attn.jsonl
bash tools/gpu_r5s.sh || exit 5
