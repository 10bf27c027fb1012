#!/bin/bash
# per-kernel decode profiles: B=1 (deferred norm vs full-row norm-in), B=8
set -o pipefail
mkdir -p gpurun_out
tools/prof_bench.sh llama3-8b 1 b1_defer || exit $?
ILLM_DEFER_NORM=0 tools/prof_bench.sh llama3-8b 1 b1_nodefer || exit $?
tools/prof_bench.sh llama3-8b 8 b8 || exit $?
head -14 gpurun_out/prof_b1_defer_decode.txt | cut -c1-160
head -14 gpurun_out/prof_b1_nodefer_decode.txt | cut -c1-160
head -16 gpurun_out/prof_b8_decode.txt | cut -c1-160
