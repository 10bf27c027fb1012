#!/bin/bash
# rocprofv3 kernel summary of the B=1 decode bench (GPU box); extra env via "$@" (VAR=val ...)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
for kv in "$@"; do export "$kv"; done
export BENCH_BATCH=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_q" -o run -- python3 "$R/bench.py" --steps 32 --warmup 4 > "$R/gpurun_out/prof_q.log" 2>&1
cd "$R"
db=$(find gpurun_out/prof_q -name "*.db" | head -1)
python3 tools/prof_summary.py "$db" 30 --after dequantize_tiled > gpurun_out/prof_q_summary.txt 2>&1 || python3 tools/prof_summary.py "$db" 30 > gpurun_out/prof_q_summary.txt
rm -rf gpurun_out/prof_q
head -20 gpurun_out/prof_q_summary.txt | cut -c1-150
