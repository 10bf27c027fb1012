#!/bin/bash
# round 5: decode knob sweep on the current kernels (B=8 / B=1), one bench process per setting
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
: > gpurun_out/r5o_sweep.jsonl
run() {  # B, label, env...
  local B=$1 lab=$2; shift 2
  env "$@" BENCH_BATCH=$B timeout -k 10 200 python bench.py --steps 64 --warmup 8 --no-tp-side > gpurun_out/r5o_tmp.log 2>&1 || { tail -5 gpurun_out/r5o_tmp.log; return 1; }
  tail -1 gpurun_out/r5o_tmp.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(json.dumps({'B': $B, 'cfg': '$lab', 'tok_s': d['value'], 'ms': d['ms_per_step']}))" | tee -a gpurun_out/r5o_sweep.jsonl
}
run 8 base X=0 || exit 3
run 8 mlp_acc ILLM_DEFER_MLP_ACC=1 || exit 3
run 8 defer_glu8 ILLM_DEFER_GLU_MAX_M=8 || exit 3
run 8 oproj_combine ILLM_OPROJ_COMBINE=1 || exit 3
run 8 v3nw8 ILLM_ATTN_V3_NW=8 || exit 3
run 8 v3off ILLM_ATTN_V3=0 || exit 3
run 8 rope_in8 ILLM_ROPE_IN_MAX_M=8 || exit 3
run 1 base X=0 || exit 3
run 1 oproj_combine ILLM_OPROJ_COMBINE=1 || exit 3
run 1 v3off ILLM_ATTN_V3=0 || exit 3
run 1 v3nw8 ILLM_ATTN_V3_NW=8 || exit 3
