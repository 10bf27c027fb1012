#!/bin/bash
# KW/NW/KS sweep of the v5 GEMV on Llama-3-70B shapes (GPU box): gpurun_out/sweep70.log
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/sweep70.log
: > $L
export GEMV_SHAPES=70b
timeout -k 10 120 python tools/gemv_sweep5.py ${1:-1,8} >> $L 2>&1 || exit $?
for nw in 4 8; do for kw in 1 2 4; do
  [ $kw -gt $nw ] && continue
  ILLM_GEMV5_NW=$nw ILLM_GEMV5_KW=$kw timeout -k 10 120 python tools/gemv_sweep5.py ${1:-1,8} glu >> $L 2>&1 || exit $?
done; done
for nw in 4 8; do for ks in 4 8 16 32; do
  ILLM_GEMV5_NW=$nw ILLM_GEMV5_KS=$ks timeout -k 10 120 python tools/gemv_sweep5.py ${1:-1,8} qkv,o,down >> $L 2>&1 || exit $?
done; done
grep -c us $L
