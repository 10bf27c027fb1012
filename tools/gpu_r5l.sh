#!/bin/bash
# round 5: library-GEMM check -- rocprof of a 1024-token prefill (B=1 and B=8 first token) and of QLoRA steps
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
BENCH_BATCH=1 timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/prof_pf1" -o run -- python3 "$R/bench.py" --steps 8 --warmup 2 --no-tp-side > "$R/gpurun_out/r5l_pf1.log" 2>&1 || exit 3
BENCH_BATCH=8 timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/prof_pf8" -o run -- python3 "$R/bench.py" --steps 8 --warmup 2 --no-tp-side > "$R/gpurun_out/r5l_pf8.log" 2>&1 || exit 4
timeout -k 10 400 rocprofv3 --kernel-trace -d "$R/gpurun_out/prof_ql" -o run -- python3 "$R/tools/bench_qlora.py" --steps 3 --warmup 1 > "$R/gpurun_out/r5l_ql.log" 2>&1 || exit 5
cd "$R"
for p in pf1 pf8 ql; do
  db=$(find gpurun_out/prof_$p -name "*.db" | head -1)
  python3 tools/prof_summary.py "$db" 40 > gpurun_out/r5l_${p}_summary.txt 2>&1
  echo "== $p: Cijk dispatches: $(grep -c Cijk gpurun_out/r5l_${p}_summary.txt)"
  head -14 gpurun_out/r5l_${p}_summary.txt | cut -c1-200
  rm -rf gpurun_out/prof_$p
done
