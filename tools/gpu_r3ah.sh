#!/bin/bash
# fused act * up (HF gated MLP) fwd + bwd: tests + QLoRA step A/B (ILLM_TRAIN_ROPE=0: HF rope)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_training.py tests/test_gpu_families.py tests/test_gpu_misc.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pt_r3ah.log 2>&1
rc=$?; tail -2 gpurun_out/pt_r3ah.log; [ $rc -ne 0 ] && exit $rc
for cfg in "1 0" "0 0" "1 40" "1 0"; do
  set -- $cfg
  ILLM_TRAIN_MLP=$1 ILLM_PREFILL_DENSE_GB=$2 timeout -k 10 400 python tools/bench_qlora.py --steps 8 --warmup 2 > gpurun_out/qlora_m$1_gb$2.log 2>&1 || exit $?
  echo "hip_mlp=$1 shadow_gb=$2 $(tail -1 gpurun_out/qlora_m$1_gb$2.log | grep -o '"ms_per_step": [0-9.]*\|"loss_last": [0-9.]*' | tr '\n' ' ')"
done
