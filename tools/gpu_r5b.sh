#!/bin/bash
# round 5: decode attention cold vs Infinity-Cache-hot KV, kernel split (rocprofv3)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
: > gpurun_out/r5b_attn.jsonl
for B in 1 8; do
  for cfg in "ILLM_ATTN_V3=0" "ILLM_ATTN_V3_NW=4" "ILLM_ATTN_V3_NW=4 ILLM_ATTN_V3_FUSE=1"; do
    env $cfg timeout -k 10 120 python tools/bench_attn_dec.py $B 1025 20 1 >> gpurun_out/r5b_attn.jsonl 2>> gpurun_out/r5b_attn.err || exit 2
  done
done
cat gpurun_out/r5b_attn.jsonl
cd /tmp && export TMPDIR=/tmp
for cfg in v2 v3; do
  if [ $cfg = v2 ]; then export ILLM_ATTN_V3=0; else export ILLM_ATTN_V3=1 ILLM_ATTN_V3_NW=4; fi
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r5b_prof_$cfg" -o run -- python3 "$R/tools/bench_attn_dec.py" 8 1025 10 32 > "$R/gpurun_out/r5b_prof_$cfg.log" 2>&1 || exit 3
  db=$(find "$R/gpurun_out/r5b_prof_$cfg" -name "*.db" | head -1)
  python3 "$R/tools/prof_summary.py" "$db" 12 > "$R/gpurun_out/r5b_${cfg}_summary.txt" 2>&1
  rm -rf "$R/gpurun_out/r5b_prof_$cfg"
done
cat "$R"/gpurun_out/r5b_v2_summary.txt "$R"/gpurun_out/r5b_v3_summary.txt
