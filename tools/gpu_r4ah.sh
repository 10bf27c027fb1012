#!/bin/bash
# round-4: the bounds / device-debug-build tests with the rebuilt _C_debug.so
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -q -rs --timeout 200 --timeout-method thread tests/test_gpu_bounds.py -m gpu > gpurun_out/t_r4ah.log 2>&1
rc=$?; tail -5 gpurun_out/t_r4ah.log; exit $rc
