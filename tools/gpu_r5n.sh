#!/bin/bash
# round 5: fused-CE vocab-sliced grad + fp8 split-K tests, QLoRA peak memory, fp8 GEMM sweep vs torch._scaled_mm
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_train_kernels.py tests/test_gpu_training.py tests/test_gpu_fp8.py tests/test_gpu_gemm8p.py -q -x --timeout 200 --timeout-method thread > gpurun_out/r5n_tests.log 2>&1 || { tail -40 gpurun_out/r5n_tests.log; exit 2; }
tail -1 gpurun_out/r5n_tests.log
timeout -k 10 400 python -u tools/bench_qlora.py --steps 6 --warmup 2 > gpurun_out/r5n_qlora.log 2>&1 || { tail -20 gpurun_out/r5n_qlora.log; exit 5; }
tail -1 gpurun_out/r5n_qlora.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print("qlora", d["ms_per_step"], d["peak_mem_gb"], d["loss_last"])'
timeout -k 10 400 python -u tools/fp8_gemm_bench.py > gpurun_out/r5n_fp8.jsonl 2> gpurun_out/r5n_fp8.err || exit 6
grep -v amdgpu gpurun_out/r5n_fp8.jsonl | python3 -c '
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d["M"], d["proj"], "kernel", d["fp8_8p_kernel_only_us"], "sm", d["fp8_scaled_mm_us"], "k/sm", d["kernel_vs_scaled_mm"])'
