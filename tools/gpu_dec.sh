#!/bin/bash
# GPU box: decode-attention tests, B=1/B=8 bench, rocprofv3 decode kernel summaries
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "attn or decode or combine or rope or gemma or softcap or alibi or engine" > gpurun_out/pt_dec.log 2>&1 || { tail -30 gpurun_out/pt_dec.log; exit 1; }
tail -1 gpurun_out/pt_dec.log
BENCH_BATCH=1 timeout -k 10 300 python bench.py --steps 64 --warmup 8 > gpurun_out/bench_b1.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 64 --warmup 8 > gpurun_out/bench_b8.log 2>&1 || exit $?
tail -1 gpurun_out/bench_b1.log | grep -o '"ms_per_step": [0-9.]*\|"first_token_latency_ms": [0-9.]*' | tr '\n' ' '; echo
tail -1 gpurun_out/bench_b8.log | grep -o '"ms_per_step": [0-9.]*\|"first_token_latency_ms": [0-9.]*' | tr '\n' ' '; echo
bash tools/prof_decode.sh > /dev/null 2>&1 || exit 1
grep "attn\|combine\|kernel time" gpurun_out/prof_b1_summary.txt | cut -c1-110
grep "attn\|combine\|kernel time" gpurun_out/prof_b8_summary.txt | cut -c1-110
