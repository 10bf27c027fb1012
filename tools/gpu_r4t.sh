#!/bin/bash
# round-4: graph-captured prefill: parity test, then bench B=1 / B=8 (prefill graph vs eager, same box)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T="timeout -k 10"
$T 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_model.py > gpurun_out/t_r4t.log 2>&1
rc=$?; tail -3 gpurun_out/t_r4t.log; [ $rc -eq 0 ] || exit $rc
for B in 1 8; do
  BENCH_BATCH=$B $T 200 python bench.py --steps 32 --warmup 4 > gpurun_out/bench_b${B}_pfg.log 2>&1 || exit $?
  BENCH_BATCH=$B $T 200 python bench.py --steps 32 --warmup 4 --no-prefill-graph > gpurun_out/bench_b${B}_pfe.log 2>&1 || exit $?
  for v in pfg pfe; do echo "B=$B $v $(grep -o '"first_token_latency_ms": [0-9.]*' gpurun_out/bench_b${B}_$v.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_b${B}_$v.log)"; done
done
