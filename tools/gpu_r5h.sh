#!/bin/bash
# round 5: GEMM / dense-GEMV / training tests, slab split-K sweep, bench B=8 / B=1 (shadow-free prefill), QLoRA step
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_gemm8p.py tests/test_gpu_dense_gemv.py tests/test_gpu_training.py "tests/test_gpu_kernels.py" -k "not test_gpu_kernels or gemv_rope or v3_variants or dequantize_device or dense_glu" -q -x --timeout 280 --timeout-method thread > gpurun_out/r5h_tests.log 2>&1 || { tail -40 gpurun_out/r5h_tests.log; exit 2; }
tail -2 gpurun_out/r5h_tests.log
timeout -k 10 300 python -u tools/bench_g8.py sym_int4 --m 8192,1024 --dense > gpurun_out/r5h_g8d.jsonl 2> gpurun_out/r5h_g8d.err || exit 3
echo "g8d ok"
for B in 8 1; do
  BENCH_BATCH=$B timeout -k 10 300 python bench.py --steps 64 --warmup 8 > gpurun_out/r5h_bench_b$B.log 2>&1 || exit 4
  echo "B=$B: $(tail -1 gpurun_out/r5h_bench_b$B.log | cut -c1-600)"
done
timeout -k 10 400 python -u tools/bench_qlora.py --steps 6 --warmup 2 > gpurun_out/r5h_qlora.log 2>&1 || { tail -20 gpurun_out/r5h_qlora.log; exit 5; }
tail -1 gpurun_out/r5h_qlora.log
