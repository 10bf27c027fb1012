#!/bin/bash
# round-4: decode B=8 / B=1 kernel traces (per-dispatch grids -> per-projection times)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for b in 8 1; do
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/prof_b$b -o run -- python3 $R/bench.py --batch $b --steps 10 --warmup 2 > $R/gpurun_out/prof_r4x_b$b.log 2>&1 || exit $?
  cd $R && python3 tools/decode_trace_summary.py /tmp/prof_b$b/run_results.db 5 > gpurun_out/decode_trace_b${b}_r4.txt 2>&1 || exit $?
  head -30 gpurun_out/decode_trace_b${b}_r4.txt
done
