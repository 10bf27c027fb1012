#!/bin/bash
# GPU box: glu tests, prefill GEMM fused-vs-library sweep, in-model A/B of the library path
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "glu or gemm" > gpurun_out/pt_glu.log 2>&1 || { tail -30 gpurun_out/pt_glu.log; exit 1; }
tail -1 gpurun_out/pt_glu.log
GEMM_M=256,512,768,1024 timeout -k 10 300 python tools/bench_prefill_gemm.py > gpurun_out/gemm_sweep.jsonl 2>&1 || exit 1
grep '"M"' gpurun_out/gemm_sweep.jsonl | cut -c1-120
bash tools/ab_env.sh ILLM_GEMM_LIB "0 1"
