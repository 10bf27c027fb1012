#!/bin/bash
# round-3 checkpoint: full GPU suite, smoke, headline bench (B=8 default) + B=1, decode profiles
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pt_full.log 2>&1
rc=$?; tail -3 gpurun_out/pt_full.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py --steps 64 --warmup 8 > gpurun_out/bench_head.log 2>&1 || exit $?
tail -1 gpurun_out/bench_head.log | cut -c1-300
BENCH_BATCH=1 timeout -k 10 300 python bench.py --steps 64 --warmup 8 > gpurun_out/bench_b1.log 2>&1 || exit $?
tail -1 gpurun_out/bench_b1.log | cut -c1-300
tools/prof_bench.sh llama3-8b 1 b1_final || exit $?
tools/prof_bench.sh llama3-8b 8 b8_final || exit $?
head -12 gpurun_out/prof_b1_final_decode.txt | cut -c1-150
head -12 gpurun_out/prof_b8_final_decode.txt | cut -c1-150
