#!/bin/bash
# GEMV ablations (production geometry), decode-attention PMC, B=8 A/B
set -o pipefail
mkdir -p gpurun_out
for a in 0 1 3 7; do
  PROBE_MODE=a timeout -k 10 120 tools/probe/gemv5_probe_a$a >> gpurun_out/gemv5_abl2.jsonl 2>&1 || exit $?
done
tools/pmc_attn_dec.sh 1 1024 1 > /dev/null || exit $?
tools/pmc_attn_dec.sh 8 1024 0 > /dev/null || exit $?
for i in 1 2; do
  BENCH_BATCH=8 timeout -k 10 300 python bench.py --steps 64 --warmup 4 > gpurun_out/ab8_hyb_$i.log 2>&1 || exit $?
  tail -1 gpurun_out/ab8_hyb_$i.log | grep -o '"ms_per_step": [0-9.]*'
  ILLM_DEFER_MAX_M=4 BENCH_BATCH=8 timeout -k 10 300 python bench.py --steps 64 --warmup 4 > gpurun_out/ab8_old_$i.log 2>&1 || exit $?
  tail -1 gpurun_out/ab8_old_$i.log | grep -o '"ms_per_step": [0-9.]*'
done
