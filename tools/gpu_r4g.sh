#!/bin/bash
# round-4: fp8 on the 8-phase GEMM (tests + sweep vs _scaled_mm), 8p GLU test
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T="timeout -k 10"
$T 300 python -u -m pytest -q -rf --timeout 120 --timeout-method thread tests/test_gpu_fp8.py tests/test_gpu_gemm8p.py > gpurun_out/t_r4g.log 2>&1
rc=$?; tail -12 gpurun_out/t_r4g.log
case $rc in 0|1) ;; *) echo "pytest rc=$rc: stopping"; exit $rc;; esac
$T 400 python -u tools/fp8_gemm_bench.py > gpurun_out/fp8_sweep_r4g.jsonl 2>&1
rc=$?; cat gpurun_out/fp8_sweep_r4g.jsonl; exit $rc
