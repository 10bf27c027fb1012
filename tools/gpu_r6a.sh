#!/bin/bash
# round 6: o_proj norm-out epilogue (gemv_accum_norm + gemv_glu_ss): kernel tests,
# decode parity, bench A/B (ILLM_ONORM=1/0) at B = 8, B = 1 sanity, decode trace B = 8
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "accum_norm or onorm or norm_in or accum_and_zeroing or glu" > gpurun_out/r6a_pytest.log 2>&1 || { tail -40 gpurun_out/r6a_pytest.log; exit 2; }
tail -2 gpurun_out/r6a_pytest.log
: > gpurun_out/r6a_ab.jsonl
run() {  # B, flag
  ILLM_ONORM=$2 BENCH_BATCH=$1 timeout -k 10 200 python bench.py --steps 64 --warmup 8 --no-tp-side > gpurun_out/r6a_tmp.log 2>&1 || { tail -5 gpurun_out/r6a_tmp.log; return 1; }
  tail -1 gpurun_out/r6a_tmp.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(json.dumps({'B': $1, 'onorm': $2, 'tok_s': d['value'], 'ms': d['ms_per_step'], 'ftl': d['first_token_latency_ms']}))" | tee -a gpurun_out/r6a_ab.jsonl
}
for i in 1 2; do
  for fl in 1 0; do run 8 $fl || exit 3; done
done
run 1 1 || exit 3
BENCH_BATCH=8 timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/prof_a8" -o run -- python3 "$R/bench.py" --steps 32 --warmup 4 --no-tp-side > "$R/gpurun_out/r6a_prof8.log" 2>&1 || exit 5
db=$(find gpurun_out/prof_a8 -name "*.db" | head -1)
python3 tools/decode_trace_summary.py "$db" 5 > gpurun_out/r6a_trace_b8.txt 2>&1 || exit 6
rm -rf gpurun_out/prof_a8
head -10 gpurun_out/r6a_trace_b8.txt
