#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_families.py tests/test_gpu_moe.py tests/test_gpu_model.py -x -v --timeout 200 --timeout-method thread > gpurun_out/pt_r3d.log 2>&1
rc=$?
tail -5 gpurun_out/pt_r3d.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r3d.log 2>&1 || exit $?
tail -2 gpurun_out/smoke_r3d.log
