#!/bin/bash
# round 5: full-K (no split) o / qkv GEMVs at M = 1 / 8 over in-workgroup K splits
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
: > gpurun_out/r5s_sweep.jsonl
for cfg in "ILLM_GEMV5_KW=1 ILLM_GEMV5_NW=4" "ILLM_GEMV5_KW=2 ILLM_GEMV5_NW=4" "ILLM_GEMV5_KW=4 ILLM_GEMV5_NW=4" \
           "ILLM_GEMV5_KW=2 ILLM_GEMV5_NW=8" "ILLM_GEMV5_KW=4 ILLM_GEMV5_NW=8"; do
  echo "# store1 $cfg" >> gpurun_out/r5s_sweep.jsonl
  env $cfg GEMV_STORE1=1 timeout -k 10 200 python tools/gemv_sweep5.py 1,8 qkv,o >> gpurun_out/r5s_sweep.jsonl 2>> gpurun_out/r5s_sweep.err || exit 2
done
echo "# acc default" >> gpurun_out/r5s_sweep.jsonl
GEMV_ACC=1 timeout -k 10 200 python tools/gemv_sweep5.py 1,8 qkv,o >> gpurun_out/r5s_sweep.jsonl 2>> gpurun_out/r5s_sweep.err || exit 3
cat gpurun_out/r5s_sweep.jsonl
