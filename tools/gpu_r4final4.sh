#!/bin/bash
# round-4: the whole GPU test suite (as the driver runs it), smoke, headline bench B=1 / B=8
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T="timeout -k 10"
$T 900 python -u -m pytest tests/ -m gpu -q -rf --timeout 180 --timeout-method thread > gpurun_out/t_r4final4.log 2>&1
rc=$?; tail -25 gpurun_out/t_r4final4.log
case $rc in 0|1) ;; *) echo "pytest rc=$rc: stopping"; exit $rc;; esac
$T 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r4final4.log 2>&1 || { tail -20 gpurun_out/smoke_r4final4.log; exit 1; }
tail -1 gpurun_out/smoke_r4final4.log
BENCH_BATCH=1 $T 200 python bench.py --steps 64 --warmup 8 > gpurun_out/bench_b1_r4final4.log 2>&1 || exit $?
$T 200 python bench.py --steps 64 --warmup 8 > gpurun_out/bench_b8_r4final4.log 2>&1 || exit $?
tail -1 gpurun_out/bench_b1_r4final4.log | cut -c1-330; tail -1 gpurun_out/bench_b8_r4final4.log | cut -c1-330
exit $rc
