#!/bin/bash
# Debug pass of the GPU tests: every kernel launch serialised and
# synchronous (AMD_SERIALIZE_KERNEL=3, HIP_LAUNCH_BLOCKING=1) so a faulting or
# racing kernel is pinned to the test that launched it.  Usage (GPU box):
#   bash tools/gpu_debug_run.sh [pytest -k expression]
set -o pipefail
mkdir -p gpurun_out
K=${1:-""}
export AMD_SERIALIZE_KERNEL=3 HIP_LAUNCH_BLOCKING=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${K:+-k "$K"} \
  > gpurun_out/pytest_gpu_serialized.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu_serialized.log
exit $rc
