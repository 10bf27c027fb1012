#!/bin/bash
# rocprofv3 kernel summary of B=1 decode at a long prompt (GPU box): tools/prof_longctx.sh [P]
set -e
P=${1:-32768}
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
BENCH_BATCH=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_p$P" -o run -- python3 "$R/bench.py" --steps 16 --warmup 2 --prompt-len $P > "$R/gpurun_out/prof_p$P.log" 2>&1
cd "$R"
db=$(find "gpurun_out/prof_p$P" -name "*.db" | head -1)
python3 tools/prof_summary.py "$db" 25 --after attn_prefill > "gpurun_out/prof_p${P}_decode.txt" 2>&1
rm -rf "gpurun_out/prof_p$P"
head -12 "gpurun_out/prof_p${P}_decode.txt"
