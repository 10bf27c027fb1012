#!/bin/bash
# round 6: prefill library-GEMM A/B (ILLM_GEMM_G8D=0: dequantize + hipBLASLt) and the
# other BASELINE models (Mixtral-8x7B, Llama-3-70B) on the round-6 kernels
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
: > gpurun_out/r6n.jsonl
run() {  # tag, env..., -- bench args
  local tag=$1; shift
  env "$@" timeout -k 10 600 python bench.py $BARGS > gpurun_out/r6n_tmp.log 2>&1 || { tail -5 gpurun_out/r6n_tmp.log; return 1; }
  tail -1 gpurun_out/r6n_tmp.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(json.dumps({'tag': '$tag', 'model': d['config']['model'], 'B': d['config']['global_batch'], 'tok_s': d['value'], 'ms': d['ms_per_step'], 'ftl': d['first_token_latency_ms']}))" | tee -a gpurun_out/r6n.jsonl
}
for i in 1 2; do for B in 8 1; do
  BARGS="--batch $B" run g8d ILLM_GEMM_G8D=1 || exit 2
  BARGS="--batch $B" run lib ILLM_GEMM_G8D=0 || exit 2
done; done
for m in mixtral-8x7b llama3-70b; do for B in 1 8; do
  BARGS="--model $m --batch $B --steps 32" run r6 X=1 || exit 3
done; done
