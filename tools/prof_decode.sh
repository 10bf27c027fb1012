#!/bin/bash
# rocprofv3 kernel trace of the B=1 and B=8 decode benchmark (GPU box).
# usage (from the repo root): bash tools/prof_decode.sh
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
export BENCH_BATCH=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_b1" -o run -- python3 "$R/bench.py" --steps 32 --warmup 4 > "$R/gpurun_out/prof_b1.log" 2>&1
export BENCH_BATCH=8
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_b8" -o run -- python3 "$R/bench.py" --steps 32 --warmup 4 > "$R/gpurun_out/prof_b8.log" 2>&1
cd "$R"
for b in b1 b8; do
  db=$(find "gpurun_out/prof_$b" -name "*.db" | head -1)
  python3 tools/prof_summary.py "$db" 40 --after attn_prefill > "gpurun_out/prof_${b}_summary.txt" 2>&1 || python3 tools/prof_summary.py "$db" 40 > "gpurun_out/prof_${b}_summary.txt"
done
tail -1 gpurun_out/prof_b1.log | cut -c1-200
# keep the summaries + rocprofv3 --stats CSVs, drop the (large) trace databases
for b in b1 b8; do
  find "gpurun_out/prof_$b" -name "*kernel_stats.csv" -exec cp {} "gpurun_out/prof_${b}_kernel_stats.csv" \;
  rm -rf "gpurun_out/prof_$b"
done
