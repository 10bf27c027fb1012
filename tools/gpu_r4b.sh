#!/bin/bash
# round-4 GPU step: engine + training-kernel tests, GEMM sweep, QLoRA step
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T="timeout -k 10"
$T 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_mfgemm.py tests/test_gpu_train_kernels.py > gpurun_out/t_r4b.log 2>&1
rc=$?; tail -15 gpurun_out/t_r4b.log; [ $rc -eq 0 ] || exit $rc
GEMM_M=1024,4096 $T 200 python -u tools/bench_mfgemm.py > gpurun_out/mfg_sweep_r4b.jsonl 2>&1 || exit 1
cat gpurun_out/mfg_sweep_r4b.jsonl
$T 300 python -u tools/bench_qlora.py --steps 5 --warmup 2 > gpurun_out/qlora_r4b.json 2>&1; tail -3 gpurun_out/qlora_r4b.json
