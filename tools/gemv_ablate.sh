#!/bin/bash
set -e
mkdir -p gpurun_out
for a in 0 1 2 3; do
  ILLM_GEMV_ABL=$a timeout -k 10 200 python tools/bench_kernels.py --m 1,8 --only gemv > gpurun_out/abl_$a.log 2>&1
done
