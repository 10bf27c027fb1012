#!/bin/bash
# device-side bounds checks (seq-len / token / decode-advance) + ILLM_DEVICE_DEBUG build, kernel + model tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_bounds.py tests/test_gpu_kernels.py tests/test_gpu_model.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pt_r3aa.log 2>&1
rc=$?; tail -3 gpurun_out/pt_r3aa.log; grep -E "PASS|FAIL|SKIP" gpurun_out/pt_r3aa.log | grep bounds; exit $rc
