#!/bin/bash
# decode attention at B=4/8: late-V vs up-front V loads with the MFMA P V form (same box A/B)
set -o pipefail
mkdir -p gpurun_out
for b in 8 4; do
  for cfg in "-1 -1" "0 -1" "0 2" "-1 -1" "0 -1"; do
    set -- $cfg
    env ILLM_ATTN_LATEV=$1 ILLM_ATTN_NWV=$2 BENCH_BATCH=$b timeout -k 10 300 python bench.py --steps 96 --warmup 4 > gpurun_out/ab_lv$1_nw$2_b$b.log 2>&1 || exit $?
    echo "b=$b latev=$1 nwv=$2 $(tail -1 gpurun_out/ab_lv$1_nw$2_b$b.log | grep -o '"ms_per_step": [0-9.]*')"
  done
done
