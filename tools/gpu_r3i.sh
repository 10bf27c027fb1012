#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_dense_gemv.py tests/test_gpu_speculative.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pt_r3h.log 2>&1
rc=$?
tail -3 gpurun_out/pt_r3h.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u tools/spec_bench.py > gpurun_out/spec_bench2.jsonl 2> gpurun_out/spec_bench2.err || exit $?
cat gpurun_out/spec_bench2.jsonl
for b in 1 8; do
  BENCH_BATCH=$b timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/ab_base_b$b.log 2>&1 || exit $?
  tail -1 gpurun_out/ab_base_b$b.log | cut -c1-200
  ILLM_ATTN_FUSED_COMBINE=1 BENCH_BATCH=$b timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/ab_fc_b$b.log 2>&1 || exit $?
  tail -1 gpurun_out/ab_fc_b$b.log | cut -c1-200
done
