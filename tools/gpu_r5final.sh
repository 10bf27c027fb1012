#!/bin/bash
# round 5 final: GPU suite, smoke, bench B = 8 / 1, decode trace at B = 8
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/final_pytest.log 2>&1 || { tail -40 gpurun_out/final_pytest.log; exit 2; }
tail -2 gpurun_out/final_pytest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final_smoke.log 2>&1 || { tail -20 gpurun_out/final_smoke.log; exit 3; }
tail -1 gpurun_out/final_smoke.log
for B in 8 1 8 1; do
  BENCH_BATCH=$B timeout -k 10 200 python bench.py --steps 64 --warmup 8 > gpurun_out/final_b$B.log 2>&1 || { tail -5 gpurun_out/final_b$B.log; exit 4; }
  tail -1 gpurun_out/final_b$B.log >> gpurun_out/final_bench.jsonl
  echo "B=$B $(tail -1 gpurun_out/final_b$B.log | grep -o '"ms_per_step": [0-9.]*') $(tail -1 gpurun_out/final_b$B.log | grep -o '"first_token_latency_ms": [0-9.]*')"
done
BENCH_BATCH=8 timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/prof_f8" -o run -- python3 "$R/bench.py" --steps 32 --warmup 4 --no-tp-side > "$R/gpurun_out/final_prof8.log" 2>&1 || exit 5
db=$(find gpurun_out/prof_f8 -name "*.db" | head -1)
python3 tools/decode_trace_summary.py "$db" 5 > gpurun_out/final_trace_b8.txt 2>&1 || exit 6
rm -rf gpurun_out/prof_f8
head -9 gpurun_out/final_trace_b8.txt
