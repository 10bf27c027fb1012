#!/bin/bash
# round 6: in-LDS low-bit 8-phase kernel as a measured prefill candidate -- tests, choices, bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_prodshape.py tests/test_gpu_gemm8p.py -k "dispatch or llama3 or lowbit or g8" -x -q --timeout 300 --timeout-method thread > gpurun_out/r6t_pytest.log 2>&1 || { tail -30 gpurun_out/r6t_pytest.log; exit 2; }
tail -1 gpurun_out/r6t_pytest.log
: > gpurun_out/r6t.jsonl
for i in 1 2; do for B in 1 8; do
  ILLM_GEMM_AUTOTUNE_LOG=1 timeout -k 10 400 python bench.py --batch $B > gpurun_out/r6t_tmp.log 2>&1 || { tail -5 gpurun_out/r6t_tmp.log; exit 3; }
  [ $i = 1 ] && grep "^\[gemm\]" gpurun_out/r6t_tmp.log > gpurun_out/prefill_choices_b${B}_r6.txt
  tail -1 gpurun_out/r6t_tmp.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(json.dumps({'B': $B, 'tok_s': d['value'], 'ms': d['ms_per_step'], 'ftl': d['first_token_latency_ms']}))" | tee -a gpurun_out/r6t.jsonl
done; done
cat gpurun_out/prefill_choices_b1_r6.txt gpurun_out/prefill_choices_b8_r6.txt
