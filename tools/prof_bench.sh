#!/bin/bash
# rocprofv3 kernel trace of bench.py decode for one model (GPU box):
#   tools/prof_bench.sh <model> <batch> [tag]
# leaves gpurun_out/prof_<tag>_summary.txt (per-kernel time over the timed
# decode steps) and the kernel_stats csv; the raw db is removed (>64 MiB).
set -e
M=${1:-llama3-8b}; B=${2:-1}; TAG=${3:-${M}_b${B}}
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$TAG" -o run -- python3 "$R/bench.py" \
  --model "$M" --batch "$B" --steps 16 --warmup 2 > "$R/gpurun_out/prof_$TAG.log" 2>&1
cd "$R"
db=$(find "gpurun_out/prof_$TAG" -name "*.db" | head -1)
python3 tools/prof_summary.py "$db" 30 > "gpurun_out/prof_${TAG}_summary.txt" 2>&1
python3 tools/prof_summary.py "$db" 30 --after attn_prefill > "gpurun_out/prof_${TAG}_decode.txt" 2>&1
find "gpurun_out/prof_$TAG" -name "*kernel_stats.csv" -exec cp {} "gpurun_out/prof_${TAG}_kernel_stats.csv" \;
rm -rf "gpurun_out/prof_$TAG"
