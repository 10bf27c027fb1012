#!/bin/bash
# Same-box A/B of two builds of the native library (GPU box):
#   tools/ab_lib.sh _C_base.so [pytest -k expr]
# alternates the default _C.so and the tagged library on the B=1 / B=8 decode bench
set -o pipefail
mkdir -p gpurun_out
ALT=$1; K=$2
if [ -n "$K" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$K" > gpurun_out/pytest_ab.log 2>&1 || { tail -30 gpurun_out/pytest_ab.log; exit 1; }
  tail -1 gpurun_out/pytest_ab.log
fi
for rep in 1 2; do for b in 1 8; do for lib in _C.so $ALT; do
  IPEX_LLM_AMD_LIB=$lib BENCH_BATCH=$b timeout -k 10 300 python bench.py --steps 256 --warmup 16 > gpurun_out/ablib.log 2>&1 || exit $?
  echo "rep=$rep B=$b lib=$lib $(tail -1 gpurun_out/ablib.log | grep -o '"ms_per_step": [0-9.]*')"
done; done; done
