#!/bin/bash
# round-4: speculative k=2 decode-window trace (busy vs span, kernels)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/prof_s -o run -- python3 $R/tools/spec_bench.py --ks 2 --skip-plain --new 64 > $R/gpurun_out/spec_trace_r4.log 2>&1 || exit $?
cd $R && tail -2 gpurun_out/spec_trace_r4.log && python3 tools/spec_trace_summary.py /tmp/prof_s/run_results.db > gpurun_out/spec_trace_summary_r4.txt 2>&1; rc=$?; head -45 gpurun_out/spec_trace_summary_r4.txt; exit $rc
