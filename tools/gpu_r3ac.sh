#!/bin/bash
# small-M prefill GEMM tiles (0 = 128x128, 6 = 128n x 64m) + QLoRA step kernel profile (dense shadow on)
set -o pipefail
mkdir -p gpurun_out
for t in 0 6; do
  ILLM_GEMM_TILE=$t GEMM_M=128,256,384,512,768 timeout -k 10 240 python tools/bench_prefill_gemm.py sym_int4 > gpurun_out/gemm_small_tile$t.jsonl 2> gpurun_out/gemm_small_tile$t.err || exit $?
  echo "tile $t"; cut -c1-100 gpurun_out/gemm_small_tile$t.jsonl
done
ILLM_PREFILL_DENSE_GB=40 bash tools/prof_qlora.sh && head -40 gpurun_out/prof_qlora_summary.txt
