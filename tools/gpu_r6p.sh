#!/bin/bash
# round 6: measured GEMM dispatch in the QLoRA step (grad_x, fused-CE head) -- tests, then
# tools/bench_qlora.py default vs ILLM_GEMM_AUTOTUNE=0, twice
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_training.py tests/test_gpu_train_kernels.py tests/test_gpu_kernels.py -k "not test_gemv_formats" -x -q --timeout 300 --timeout-method thread > gpurun_out/r6p_pytest.log 2>&1 || { tail -30 gpurun_out/r6p_pytest.log; exit 2; }
tail -2 gpurun_out/r6p_pytest.log
: > gpurun_out/r6p.jsonl
for i in 1 2; do for at in 1; do
  ILLM_GEMM_AUTOTUNE=$at ILLM_GEMM_AUTOTUNE_LOG=$([ $i = 1 ] && [ $at = 1 ] && echo 1) timeout -k 10 500 python tools/bench_qlora.py > gpurun_out/r6p_tmp.log 2>&1 || { tail -5 gpurun_out/r6p_tmp.log; exit 3; }
  [ $i = 1 ] && [ $at = 1 ] && grep "^\[gemm\]" gpurun_out/r6p_tmp.log > gpurun_out/r6p_choices.txt
  echo "{\"autotune\": $at, \"run\": $(tail -1 gpurun_out/r6p_tmp.log)}" | tee -a gpurun_out/r6p.jsonl
done; done
