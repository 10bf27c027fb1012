#!/bin/bash
# auto plan vs PF=8 and a few KW/KS points (GPU box): gpurun_out/sweep5b.log
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/sweep5b.log
timeout -k 10 120 python tools/gemv_sweep5.py 1,4,8,16 >> gpurun_out/sweep5b.log 2>&1 || exit $?
ILLM_GEMV5_PF=8 timeout -k 10 120 python tools/gemv_sweep5.py 1,4,8,16 | sed 's/"kw"/"pf": 8, "kw"/' >> gpurun_out/sweep5b.log 2>&1 || exit $?
for ks in 16 32; do ILLM_GEMV5_KS=$ks ILLM_GEMV5_KW=1 timeout -k 10 120 python tools/gemv_sweep5.py 1,8 down >> gpurun_out/sweep5b.log 2>&1 || exit $?; done
for kw in 2 4; do ILLM_GEMV5_KW=$kw timeout -k 10 120 python tools/gemv_sweep5.py 1,4,8,16 glu >> gpurun_out/sweep5b.log 2>&1 || exit $?; done
grep -c us gpurun_out/sweep5b.log
