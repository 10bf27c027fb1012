#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_fp8.py tests/test_gpu_families.py -x -v --timeout 200 --timeout-method thread > gpurun_out/pt_r3e.log 2>&1
rc=$?
tail -5 gpurun_out/pt_r3e.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/fp8_gemm_bench.py > gpurun_out/fp8_sweep.jsonl 2> gpurun_out/fp8_sweep.err || exit $?
cat gpurun_out/fp8_sweep.jsonl | cut -c1-300
