#!/bin/bash
# round-4: 4-wave 128x128-per-wave dense GEMM (gemm_4w.hip): numerics, then timing vs 8p / hipBLASLt
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T="timeout -k 10"
$T 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm8p.py > gpurun_out/t_r4l.log 2>&1
rc=$?; tail -3 gpurun_out/t_r4l.log; [ $rc -eq 0 ] || exit $rc
GEMM_M=1024,4096,8192 $T 400 python -u tools/bench_gemm8p.py > gpurun_out/g4w_sweep_r4l.jsonl 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/g4w_sweep_r4l.jsonl; exit $rc
