#!/bin/bash
# round 5: chained down -> qkv decode GEMVs: tests, bench A/B (ILLM_GEMV_CHAIN 1 / 0), B=8 decode trace
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "chain or gemv_rope or norm_in or deferred" -q -x --timeout 200 --timeout-method thread > gpurun_out/r5k_tests.log 2>&1 || { tail -40 gpurun_out/r5k_tests.log; exit 2; }
tail -1 gpurun_out/r5k_tests.log
for B in 8 1; do
  for c in 1 0; do
    ILLM_GEMV_CHAIN=$c BENCH_BATCH=$B timeout -k 10 300 python bench.py --steps 64 --warmup 8 > gpurun_out/r5k_bench_b${B}_c$c.log 2>&1 || exit 4
    echo "B=$B chain=$c: $(tail -1 gpurun_out/r5k_bench_b${B}_c$c.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["first_token_latency_ms"])')"
  done
done
cd /tmp && export TMPDIR=/tmp
BENCH_BATCH=8 timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/prof_k8" -o run -- python3 "$R/bench.py" --steps 32 --warmup 4 --no-tp-side > "$R/gpurun_out/r5k_prof8.log" 2>&1 || exit 5
cd "$R"
db=$(find gpurun_out/prof_k8 -name "*.db" | head -1)
python3 tools/decode_trace_summary.py "$db" 5 > gpurun_out/r5k_trace_b8.txt 2>&1
rm -rf gpurun_out/prof_k8
head -30 gpurun_out/r5k_trace_b8.txt
