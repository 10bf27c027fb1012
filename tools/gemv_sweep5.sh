#!/bin/bash
# KW x KS sweep of the v5 GEMV (GPU box): gpurun_out/sweep5.log
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/sweep5.log
for kw in 1 2 4; do for ks in 1 2 4 8; do
  ILLM_GEMV5_KW=$kw ILLM_GEMV5_KS=$ks timeout -k 10 120 python tools/gemv_sweep5.py ${1:-1,8} >> gpurun_out/sweep5.log 2>&1 || exit $?
done; done
timeout -k 10 120 python tools/gemv_sweep5.py ${1:-1,8} >> gpurun_out/sweep5.log 2>&1 || exit $?
grep -c us gpurun_out/sweep5.log
