#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_fp8.py tests/test_gpu_speculative.py -x -v --timeout 200 --timeout-method thread > gpurun_out/pt_r3f.log 2>&1
rc=$?
tail -5 gpurun_out/pt_r3f.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/fp8_gemm_bench.py > gpurun_out/fp8_sweep2.jsonl 2> gpurun_out/fp8_sweep2.err || exit $?
cut -c1-260 gpurun_out/fp8_sweep2.jsonl | head -8
timeout -k 10 500 python -u tools/spec_bench.py > gpurun_out/spec_bench.jsonl 2> gpurun_out/spec_bench.err || exit $?
cat gpurun_out/spec_bench.jsonl
