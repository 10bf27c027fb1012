#!/bin/bash
# round 6: the deferred-norm 8-slot GLU XM form (ILLM_GEMV5_XM_RT=3) -- numerics tests, same-box A/B at B=1
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
for rep in 1 2; do
ILLM_GEMV5_XM_RT=3 ILLM_GEMV5_TRACE=1 timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_prodshape.py -k "norm_in or llama3 or decode or graph or greedy" -x -q --timeout 300 --timeout-method thread > gpurun_out/r6v_pytest.log 2>&1 || { grep -v "^\[gemv5\]" gpurun_out/r6v_pytest.log | tail -30; exit 2; }
grep -v "^\[gemv5\]" gpurun_out/r6v_pytest.log | tail -1
done
grep -c "XM 2 XS 8 epi 2" gpurun_out/r6v_pytest.log || true
: > gpurun_out/r6v_ab.jsonl
for i in 1 2; do for rt in 3 2; do
  ILLM_GEMV5_XM_RT=$rt timeout -k 10 300 python bench.py --batch 1 > gpurun_out/r6v_tmp.log 2>&1 || { tail -5 gpurun_out/r6v_tmp.log; exit 5; }
  tail -1 gpurun_out/r6v_tmp.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(json.dumps({'xm_rt': $rt, 'B': 1, 'tok_s': d['value'], 'ms': d['ms_per_step'], 'ftl': d['first_token_latency_ms']}))" | tee -a gpurun_out/r6v_ab.jsonl
done; done
