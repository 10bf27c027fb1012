#!/bin/bash
# round 6: first-token (batched prefill) kernel breakdown, B=8 and B=1
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
for B in 8 1; do
timeout -k 10 400 rocprofv3 --kernel-trace -d "$R/gpurun_out/pprof$B" -o run -- python3 "$R/bench.py" --batch $B --steps 4 --warmup 2 > gpurun_out/r6s_$B.log 2>&1 || { tail -20 gpurun_out/r6s_$B.log; exit 2; }
db=$(find gpurun_out/pprof$B -name "*.db" | head -1)
python3 tools/kernel_summary.py "$db" reduce_kernel 3 30 > gpurun_out/prefill_kernels_b${B}_r6.txt 2>&1 || { cat gpurun_out/prefill_kernels_b${B}_r6.txt; exit 3; }
rm -rf gpurun_out/pprof$B
cut -c1-190 gpurun_out/prefill_kernels_b${B}_r6.txt | head -22
done
