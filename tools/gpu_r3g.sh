#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/fp8_gemm_bench.py > gpurun_out/fp8_sweep2.jsonl 2> gpurun_out/fp8_sweep2.err || exit $?
cut -c1-260 gpurun_out/fp8_sweep2.jsonl | head -4
timeout -k 10 600 python -u tools/spec_bench.py > gpurun_out/spec_bench.jsonl 2> gpurun_out/spec_bench.err || exit $?
cat gpurun_out/spec_bench.jsonl
