#!/bin/bash
# round 5: decode attention v3 with the fused-RoPE loads behind the K / V rows and per-mode launch bounds
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "attn or rope or decode" > gpurun_out/r5q_pytest.log 2>&1 || { tail -30 gpurun_out/r5q_pytest.log; exit 2; }
tail -2 gpurun_out/r5q_pytest.log
: > gpurun_out/r5q_attn.jsonl
for B in 1 8; do
  timeout -k 10 120 python tools/bench_attn_dec.py $B 1025 20 >> gpurun_out/r5q_attn.jsonl || exit 3
done
cat gpurun_out/r5q_attn.jsonl
for B in 8 1; do
  BENCH_BATCH=$B timeout -k 10 200 python bench.py --steps 64 --warmup 8 --no-tp-side > gpurun_out/r5q_b$B.log 2>&1 || { tail -5 gpurun_out/r5q_b$B.log; exit 4; }
  tail -1 gpurun_out/r5q_b$B.log
done
