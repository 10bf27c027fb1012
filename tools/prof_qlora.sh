#!/bin/bash
# rocprofv3 kernel trace of the QLoRA training step (GPU box).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_qlora" -o run -- python3 "$R/tools/bench_qlora.py" --steps 3 --warmup 1 > "$R/gpurun_out/prof_qlora.log" 2>&1
cd "$R"
db=$(find gpurun_out/prof_qlora -name "*.db" | head -1)
python3 tools/prof_summary.py "$db" 30 > gpurun_out/prof_qlora_summary.txt 2>&1
find gpurun_out/prof_qlora -name "*kernel_stats.csv" -exec cp {} gpurun_out/prof_qlora_kernel_stats.csv \;
rm -rf gpurun_out/prof_qlora
