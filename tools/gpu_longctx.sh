#!/bin/bash
# GPU box: RWKV-5 tests + long-context decode bench (B=1, prompts 8K / 32K)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_rwkv5.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_rwkv5.log 2>&1 || { tail -30 gpurun_out/pytest_rwkv5.log; exit 1; }
tail -3 gpurun_out/pytest_rwkv5.log
for P in ${PLENS:-8192 32768}; do
  BENCH_BATCH=1 timeout -k 10 300 python bench.py --steps 32 --warmup 4 --prompt-len $P > gpurun_out/bench_p$P.log 2>&1 || exit $?
  echo "P=$P $(tail -1 gpurun_out/bench_p$P.log | grep -o '"ms_per_step": [0-9.]*') $(tail -1 gpurun_out/bench_p$P.log | grep -o '"first_token_latency_ms": [0-9.]*')"
done
