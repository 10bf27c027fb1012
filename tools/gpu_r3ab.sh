#!/bin/bash
# prefill GEMM block shapes: 128n x 128m (default) vs 128n x 64m (more blocks on 256 CUs) vs 2x2 wave grid
set -o pipefail
mkdir -p gpurun_out
for t in 0 5 6 3; do
  ILLM_GEMM_TILE=$t GEMM_M=1024,2048,4096 timeout -k 10 240 python tools/bench_prefill_gemm.py sym_int4 > gpurun_out/gemm_tile$t.jsonl 2> gpurun_out/gemm_tile$t.err || exit $?
  echo "tile $t"; cut -c1-120 gpurun_out/gemm_tile$t.jsonl
done
