#!/bin/bash
# round 5: norm-in staging with batched weight loads; batch >= 4 atomic GEMV plan (A/B at B = 8), B = 1 check
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "norm_in or decode or gemv" > gpurun_out/r5v_pytest.log 2>&1 || { tail -30 gpurun_out/r5v_pytest.log; exit 2; }
tail -2 gpurun_out/r5v_pytest.log
: > gpurun_out/r5v_ab.jsonl
run() {  # B, label, env...
  local B=$1 lab=$2; shift 2
  env "$@" BENCH_BATCH=$B timeout -k 10 200 python bench.py --steps 64 --warmup 8 --no-tp-side > gpurun_out/r5v_tmp.log 2>&1 || { tail -5 gpurun_out/r5v_tmp.log; return 1; }
  tail -1 gpurun_out/r5v_tmp.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(json.dumps({'B': $B, 'cfg': '$lab', 'tok_s': d['value'], 'ms': d['ms_per_step'], 'ftl_ms': d['first_token_latency_ms']}))" | tee -a gpurun_out/r5v_ab.jsonl
}
for i in 1 2; do
  run 8 "glu4_plan1" ILLM_DEFER_GLU_MAX_M=4 ILLM_GEMV5_ACC_PLAN=1 || exit 3
  run 8 "glu8_plan1" ILLM_DEFER_GLU_MAX_M=8 ILLM_GEMV5_ACC_PLAN=1 || exit 3
  run 8 "glu4_plan0" ILLM_DEFER_GLU_MAX_M=4 ILLM_GEMV5_ACC_PLAN=0 || exit 3
  run 8 "glu8_plan0" ILLM_DEFER_GLU_MAX_M=8 ILLM_GEMV5_ACC_PLAN=0 || exit 3
done
run 1 "b1" X=0 || exit 3
run 1 "b1" X=0 || exit 3
