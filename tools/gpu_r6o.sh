#!/bin/bash
# round 6: measured prefill GEMM dispatch -- tests, then bench B=8 / B=1 (autotune on / off)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_prodshape.py tests/test_gpu_model.py tests/test_gpu_families.py -x -q --timeout 300 --timeout-method thread -k "dispatch or llama3 or prefill or graph or famil" > gpurun_out/r6o_pytest.log 2>&1 || { tail -30 gpurun_out/r6o_pytest.log; exit 2; }
tail -2 gpurun_out/r6o_pytest.log
: > gpurun_out/r6o.jsonl
for i in 1 2; do for B in 8 1; do for at in 1 0; do
  ILLM_GEMM_AUTOTUNE=$at timeout -k 10 400 python bench.py --batch $B > gpurun_out/r6o_tmp.log 2>&1 || { tail -5 gpurun_out/r6o_tmp.log; exit 3; }
  tail -1 gpurun_out/r6o_tmp.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(json.dumps({'autotune': $at, 'B': $B, 'tok_s': d['value'], 'ms': d['ms_per_step'], 'ftl': d['first_token_latency_ms']}))" | tee -a gpurun_out/r6o.jsonl
done; done; done
