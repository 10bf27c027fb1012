#!/bin/bash
# round-4: 4-wave GEMM numerics, speculative exactness, encoder flash attention,
# training attention regression; then GEMM timing (4w vs 8p vs hipBLASLt) and spec bench
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T="timeout -k 10"
$T 420 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_gemm8p.py tests/test_gpu_encoders.py tests/test_gpu_speculative.py tests/test_gpu_train_kernels.py > gpurun_out/t_r4l.log 2>&1
rc=$?; tail -4 gpurun_out/t_r4l.log; [ $rc -eq 0 ] || exit $rc
$T 240 python -u tools/spec_bench.py --ks 2,4,6 > gpurun_out/spec_r4l.jsonl 2>&1
rc=$?; grep mode gpurun_out/spec_r4l.jsonl; [ $rc -eq 0 ] || exit $rc
GEMM_M=1024,4096,8192 $T 300 python -u tools/bench_gemm8p.py > gpurun_out/g4w_sweep_r4l.jsonl 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/g4w_sweep_r4l.jsonl; exit $rc
