#!/bin/bash
# round 5: v3 decode attention -- numerics, per-layer timing sweep, end-to-end bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 280 --timeout-method thread \
  -k "attn_decode or rope or combine" > gpurun_out/r5a_pytest.log 2>&1 || { tail -30 gpurun_out/r5a_pytest.log; exit 1; }
tail -3 gpurun_out/r5a_pytest.log
: > gpurun_out/r5a_attn.jsonl
for B in 1 8; do
  for cfg in "ILLM_ATTN_V3=0" "ILLM_ATTN_V3_NW=2" "ILLM_ATTN_V3_NW=4" "ILLM_ATTN_V3_NW=8" \
             "ILLM_ATTN_V3_NW=2 ILLM_ATTN_V3_FUSE=1" "ILLM_ATTN_V3_NW=4 ILLM_ATTN_V3_FUSE=1" "ILLM_ATTN_V3_NW=8 ILLM_ATTN_V3_FUSE=1"; do
    env $cfg timeout -k 10 120 python tools/bench_attn_dec.py $B 1025 20 >> gpurun_out/r5a_attn.jsonl 2>> gpurun_out/r5a_attn.err || exit 2
  done
done
cat gpurun_out/r5a_attn.jsonl
for B in 1 8; do
  BENCH_BATCH=$B timeout -k 10 200 python bench.py --steps 32 --warmup 4 > gpurun_out/r5a_bench_b$B.log 2>&1 || exit 3
  ILLM_ATTN_V3=0 BENCH_BATCH=$B timeout -k 10 200 python bench.py --steps 32 --warmup 4 > gpurun_out/r5a_bench_v2_b$B.log 2>&1 || exit 3
  tail -1 gpurun_out/r5a_bench_b$B.log | cut -c1-300; tail -1 gpurun_out/r5a_bench_v2_b$B.log | cut -c1-300
done
