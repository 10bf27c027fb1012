#!/bin/bash
# round-4: speculative exactness (chunked decode attention), encoder flash attention, training attention regression
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T="timeout -k 10"
$T 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_encoders.py tests/test_gpu_speculative.py tests/test_gpu_train_kernels.py tests/test_gpu_training.py > gpurun_out/t_r4m.log 2>&1
rc=$?; tail -5 gpurun_out/t_r4m.log; [ $rc -eq 0 ] || exit $rc
$T 500 python -u tools/spec_bench.py --ks 2,4,6 > gpurun_out/spec_r4m.jsonl 2>&1
rc=$?; grep mode gpurun_out/spec_r4m.jsonl; exit $rc
