#!/bin/bash
# batch-8 deferred-norm MLP (atomic gate/up + GLU-in down): tests + A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pt_r3w.log 2>&1
rc=$?; tail -3 gpurun_out/pt_r3w.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for v in 1 0; do
    ILLM_DEFER_MLP_ACC=$v BENCH_BATCH=8 timeout -k 10 300 python bench.py --steps 64 --warmup 4 > gpurun_out/ab_mlpacc${v}_$i.log 2>&1 || exit $?
    echo "mlpacc=$v $(tail -1 gpurun_out/ab_mlpacc${v}_$i.log | grep -o '"ms_per_step": [0-9.]*')"
  done
done
