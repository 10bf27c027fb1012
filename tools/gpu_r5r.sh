#!/bin/bash
# round 5: v3 waves-per-workgroup re-sweep after the load reordering (B = 1 / 8), plus bench B = 1
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
: > gpurun_out/r5r_attn.jsonl
for nw in 2 4 8; do
  for B in 1 8; do
    ILLM_ATTN_V3_NW=$nw timeout -k 10 120 python tools/bench_attn_dec.py $B 1025 20 >> gpurun_out/r5r_attn.jsonl || exit 3
  done
done
cat gpurun_out/r5r_attn.jsonl
for i in 1 2; do
  BENCH_BATCH=1 timeout -k 10 200 python bench.py --steps 64 --warmup 8 --no-tp-side > gpurun_out/r5r_b1_$i.log 2>&1 || { tail -5 gpurun_out/r5r_b1_$i.log; exit 4; }
  tail -1 gpurun_out/r5r_b1_$i.log | grep -o '"ms_per_step": [0-9.]*'
done
