#!/bin/bash
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T="timeout -k 10"
$T 200 python -u -m pytest -q -rf --timeout 120 --timeout-method thread tests/test_gpu_fp8.py > gpurun_out/t_r4h.log 2>&1
rc=$?; tail -5 gpurun_out/t_r4h.log
case $rc in 0|1) ;; *) exit $rc;; esac
$T 400 python -u tools/fp8_gemm_bench.py > gpurun_out/fp8_sweep_r4h.jsonl 2>&1
rc=$?; cat gpurun_out/fp8_sweep_r4h.jsonl | cut -c1-400; exit $rc
