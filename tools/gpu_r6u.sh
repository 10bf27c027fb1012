#!/bin/bash
# round 6: the checked XM subset on by default -- random-input checker, numerics tests, same-box A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
timeout -k 10 200 tools/probe/xm_v2 > gpurun_out/r6u_xmcheck.log 2>&1 || { tail -5 gpurun_out/r6u_xmcheck.log; exit 2; }
grep "FAIL\|fails=" gpurun_out/r6u_xmcheck.log
grep -q "fails=0" gpurun_out/r6u_xmcheck.log || exit 3
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_prodshape.py tests/test_gpu_model.py tests/test_gpu_tp.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r6u_pytest.log 2>&1 || { tail -30 gpurun_out/r6u_pytest.log; exit 4; }
tail -1 gpurun_out/r6u_pytest.log
: > gpurun_out/r6u_ab.jsonl
for i in 1 2; do for B in 8 1; do for rt in 2 0; do
  ILLM_GEMV5_XM_RT=$rt timeout -k 10 300 python bench.py --batch $B > gpurun_out/r6u_tmp.log 2>&1 || { tail -5 gpurun_out/r6u_tmp.log; exit 5; }
  tail -1 gpurun_out/r6u_tmp.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(json.dumps({'xm_rt': $rt, 'B': $B, 'tok_s': d['value'], 'ms': d['ms_per_step'], 'ftl': d['first_token_latency_ms'], 'ids': d['sample_next_ids']}))" | tee -a gpurun_out/r6u_ab.jsonl
done; done; done
