#!/bin/bash
# round-4: QLoRA step after the in-place gxa slices + per-dispatch trace of one step (copies / fills by grid)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_training.py -m gpu > gpurun_out/t_r4aa.log 2>&1
rc=$?; tail -2 gpurun_out/t_r4aa.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/bench_qlora.py --steps 8 --warmup 2 > gpurun_out/qlora_r4aa.json 2>&1 || exit $?
grep -o '"ms_per_step": [0-9.]*' gpurun_out/qlora_r4aa.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/prof_q -o run -- python3 $R/tools/bench_qlora.py --steps 2 --warmup 1 > $R/gpurun_out/prof_r4aa.log 2>&1 || exit $?
cd $R && python3 tools/trace_by_grid.py /tmp/prof_q/run_results.db 2 > gpurun_out/qlora_trace_by_grid_r4.txt 2>&1; rc=$?; head -60 gpurun_out/qlora_trace_by_grid_r4.txt; exit $rc
