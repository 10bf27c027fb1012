#!/bin/bash
# round-4: the whole GPU test suite (as the driver runs it) + QLoRA step
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T="timeout -k 10"
$T 1000 python -u -m pytest tests/ -m gpu -q -rf --timeout 180 --timeout-method thread > gpurun_out/t_r4j.log 2>&1
rc=$?; tail -25 gpurun_out/t_r4j.log
case $rc in 0|1) ;; *) echo "pytest rc=$rc: stopping"; exit $rc;; esac
$T 200 python -u tools/bench_qlora.py --steps 4 --warmup 2 > gpurun_out/qlora_r4j.json 2>&1; tail -1 gpurun_out/qlora_r4j.json | cut -c1-200
