#!/bin/bash
# round-4 GPU step: engine / training-kernel / EP / TP tests (no -x: all
# results), GEMM sweep, QLoRA step.  Stops after a crash or a time limit.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T="timeout -k 10"
$T 600 python -u -m pytest -q -rf --timeout 120 --timeout-method thread tests/test_gpu_mfgemm.py \
  tests/test_gpu_train_kernels.py tests/test_gpu_ep.py tests/test_gpu_allreduce.py tests/test_gpu_tp.py tests/test_gpu_speculative.py -s \
  > gpurun_out/t_r4c.log 2>&1
rc=$?; tail -30 gpurun_out/t_r4c.log
case $rc in 0|1) ;; *) echo "pytest rc=$rc: stopping"; exit $rc;; esac
GEMM_M=1024,4096 $T 240 python -u tools/bench_mfgemm.py > gpurun_out/mfg_sweep_r4c.jsonl 2>&1
rc=$?; cat gpurun_out/mfg_sweep_r4c.jsonl | tail -40; [ $rc -eq 0 ] || exit $rc
$T 300 python -u tools/bench_qlora.py --steps 5 --warmup 2 > gpurun_out/qlora_r4c.json 2>&1; tail -3 gpurun_out/qlora_r4c.json
