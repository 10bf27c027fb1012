#!/bin/bash
# round-4: headline bench with the current defaults + QLoRA kernel trace (default path)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T="timeout -k 10"
$T 400 python -u bench.py --steps 64 --warmup 8 > gpurun_out/bench_r4i.json 2> gpurun_out/bench_r4i.err
rc=$?; tail -1 gpurun_out/bench_r4i.json | cut -c1-400; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_r4i.err; exit $rc; }
$T 200 python -u tools/bench_qlora.py --steps 4 --warmup 2 > gpurun_out/qlora_r4i.json 2>&1 || exit 1
tail -1 gpurun_out/qlora_r4i.json | cut -c1-200
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
$T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_qlora_r4i -o run --output-format csv -- python -u tools/bench_qlora.py --steps 2 --warmup 1 > gpurun_out/prof_qlora_r4i.log 2>&1
echo "rocprof rc=$?"
