#!/bin/bash
# rocprofv3 kernel trace of the prefill (first-token) phase of bench.py, B=1 (GPU box)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
export BENCH_BATCH=${1:-1}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_pf" -o run -- python3 "$R/bench.py" --steps 2 --warmup 1 > "$R/gpurun_out/prof_pf.log" 2>&1
cd "$R"
db=$(find gpurun_out/prof_pf -name "*.db" | head -1)
python3 tools/prof_summary.py "$db" 30 --after dequantize_tiled > gpurun_out/prof_prefill_summary.txt 2>&1 || python3 tools/prof_summary.py "$db" 30 > gpurun_out/prof_prefill_summary.txt
rm -rf gpurun_out/prof_pf
tail -1 gpurun_out/prof_pf.log | cut -c1-200
