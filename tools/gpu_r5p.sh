#!/bin/bash
# round 5: decode GEMV geometry re-sweep on the current kernels (GLU at M = 1 / 8; atomic qkv / o / down at M = 8)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
: > gpurun_out/r5p_sweep.jsonl
for cfg in "X=0" "ILLM_GEMV5_KW=1 ILLM_GEMV5_NW=4" "ILLM_GEMV5_KW=2 ILLM_GEMV5_NW=4" "ILLM_GEMV5_KW=4 ILLM_GEMV5_NW=4" \
           "ILLM_GEMV5_KW=1 ILLM_GEMV5_NW=8" "ILLM_GEMV5_KW=2 ILLM_GEMV5_NW=8" "ILLM_GEMV5_KW=4 ILLM_GEMV5_NW=8"; do
  echo "# glu $cfg" >> gpurun_out/r5p_sweep.jsonl
  env $cfg timeout -k 10 200 python tools/gemv_sweep5.py 1,8 glu >> gpurun_out/r5p_sweep.jsonl 2>> gpurun_out/r5p_sweep.err || exit 2
done
for cfg in "X=0" "ILLM_GEMV5_KS=4 ILLM_GEMV5_NW=8" "ILLM_GEMV5_KS=8 ILLM_GEMV5_NW=8" "ILLM_GEMV5_KS=16 ILLM_GEMV5_NW=8" \
           "ILLM_GEMV5_KS=4 ILLM_GEMV5_NW=4" "ILLM_GEMV5_KS=8 ILLM_GEMV5_NW=4" "ILLM_GEMV5_KS=16 ILLM_GEMV5_NW=4"; do
  echo "# acc $cfg" >> gpurun_out/r5p_sweep.jsonl
  env $cfg GEMV_ACC=1 timeout -k 10 200 python tools/gemv_sweep5.py 8 qkv,o,down >> gpurun_out/r5p_sweep.jsonl 2>> gpurun_out/r5p_sweep.err || exit 3
done
cat gpurun_out/r5p_sweep.jsonl
