#!/bin/bash
# round 5: o_proj / lm_head geometry at M = 8 (split-1 candidates for the residual epilogue / argmax epilogue)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
: > gpurun_out/r5d_sweep.jsonl
for cfg in "X=0" "ILLM_GEMV5_KS=1 ILLM_GEMV5_KW=4 ILLM_GEMV5_NW=4" "ILLM_GEMV5_KS=1 ILLM_GEMV5_KW=2 ILLM_GEMV5_NW=4" \
           "ILLM_GEMV5_KS=1 ILLM_GEMV5_KW=8 ILLM_GEMV5_NW=8" "ILLM_GEMV5_KS=1 ILLM_GEMV5_KW=4 ILLM_GEMV5_NW=8" \
           "ILLM_GEMV5_KS=2 ILLM_GEMV5_KW=4 ILLM_GEMV5_NW=8" "ILLM_GEMV5_KS=1 ILLM_GEMV5_KW=1 ILLM_GEMV5_NW=4" \
           "ILLM_GEMV5_KS=1 ILLM_GEMV5_KW=1 ILLM_GEMV5_NW=8" "ILLM_GEMV5_KS=1 ILLM_GEMV5_KW=2 ILLM_GEMV5_NW=8"; do
  echo "# $cfg" >> gpurun_out/r5d_sweep.jsonl
  env $cfg timeout -k 10 200 python tools/gemv_sweep5.py 1,8 o,lm_head >> gpurun_out/r5d_sweep.jsonl 2>> gpurun_out/r5d_sweep.err || exit 2
done
cat gpurun_out/r5d_sweep.jsonl
