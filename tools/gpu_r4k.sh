#!/bin/bash
# round-4: speculative decoding bench (generated-token agreement) + kernel trace of one k=2 run
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T="timeout -k 10"
$T 400 python -u tools/spec_bench.py --ks 2,3,4 --std 0.05 > gpurun_out/spec_r4k.jsonl 2>&1
rc=$?; cat gpurun_out/spec_r4k.jsonl | grep mode; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
$T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_spec_r4k -o run --output-format csv -- python -u tools/spec_bench.py --ks 2 --std 0.05 --skip-plain > gpurun_out/prof_spec_r4k.log 2>&1
echo "rocprof rc=$?"
