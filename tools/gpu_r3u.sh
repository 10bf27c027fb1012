#!/bin/bash
# two-wave decode attention splits: GPU tests, bench A/B (ILLM_ATTN_NWV=1/2)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_families.py tests/test_gpu_speculative.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pt_r3u.log 2>&1
rc=$?; tail -3 gpurun_out/pt_r3u.log; [ $rc -ne 0 ] && exit $rc
for b in 1 8; do
  for nw in 2 1 2 1; do
    ILLM_ATTN_NWV=$nw BENCH_BATCH=$b timeout -k 10 300 python bench.py --steps 64 --warmup 4 > gpurun_out/ab_nwv${nw}_b$b.log 2>&1 || exit $?
    echo "b=$b nwv=$nw $(tail -1 gpurun_out/ab_nwv${nw}_b$b.log | grep -o '"ms_per_step": [0-9.]*')"
  done
done
ILLM_PREFILL_DENSE_GB=40 timeout -k 10 400 python tools/bench_qlora.py --steps 6 --warmup 2 > gpurun_out/qlora_shadow.log 2>&1 || exit $?
tail -1 gpurun_out/qlora_shadow.log | cut -c1-200
