#!/bin/bash
# round-4: staggered 8-phase GEMM (dense + low-bit decode) tests and sweep
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T="timeout -k 10"
$T 300 python -u -m pytest -q -rf --timeout 120 --timeout-method thread tests/test_gpu_gemm8p.py > gpurun_out/t_r4f.log 2>&1
rc=$?; tail -12 gpurun_out/t_r4f.log
case $rc in 0|1) ;; *) echo "pytest rc=$rc: stopping"; exit $rc;; esac
GEMM_M=1024,4096,8192 GEMM_Q=dense,sym_int4,nf4 $T 400 python -u tools/bench_gemm8p.py > gpurun_out/g8p_sweep_r4f.jsonl 2>&1
rc=$?; cat gpurun_out/g8p_sweep_r4f.jsonl; exit $rc
