#!/bin/bash
# round 6: QLoRA step kernel breakdown (rocprofv3 --kernel-trace, last 3 optimizer steps)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace -d "$R/gpurun_out/qprof" -o run -- python3 "$R/tools/bench_qlora.py" --steps 4 --warmup 2 > gpurun_out/r6q.log 2>&1 || { tail -20 gpurun_out/r6q.log; exit 2; }
db=$(find gpurun_out/qprof -name "*.db" | head -1)
python3 tools/kernel_summary.py "$db" fused_adamw 3 45 > gpurun_out/qlora_kernels_r6.txt 2>&1 || { cat gpurun_out/qlora_kernels_r6.txt; exit 3; }
rm -rf gpurun_out/qprof
cat gpurun_out/qlora_kernels_r6.txt | cut -c1-200
