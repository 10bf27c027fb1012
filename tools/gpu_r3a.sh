#!/bin/bash
# round-3 A/B: v5 GEMV PF8 on/off (standalone decode shapes + B=1/B=8 bench), then the TP / all-reduce GPU tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 150 python tools/gemv_decode_ab.py 1,4,8 > gpurun_out/ab_pf0.jsonl 2>&1 || exit $?
ILLM_GEMV5_PF8=1 timeout -k 10 150 python tools/gemv_decode_ab.py 1,4,8 > gpurun_out/ab_pf8.jsonl 2>&1 || exit $?
for pf in 0 1 0 1; do
  ILLM_GEMV5_PF8=$pf BENCH_BATCH=1 timeout -k 10 200 python bench.py --steps 128 --warmup 8 > gpurun_out/b1_pf$pf.log 2>&1 || exit $?
  tail -1 gpurun_out/b1_pf$pf.log | cut -c1-220
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_allreduce.py tests/test_gpu_tp.py -x -v --timeout 200 --timeout-method thread > gpurun_out/pt_tp.log 2>&1
rc=$?
tail -5 gpurun_out/pt_tp.log
exit $rc
