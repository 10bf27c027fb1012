#!/bin/bash
# round-4: re-check the failures after the clean rebuild, QLoRA A/B of the
# new training kernels, and a kernel-trace profile of the default QLoRA step
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T="timeout -k 10"
$T 300 python -u -m pytest -q -rf --timeout 120 --timeout-method thread tests/test_gpu_mfgemm.py \
  tests/test_gpu_ep.py > gpurun_out/t_r4d.log 2>&1
rc=$?; tail -12 gpurun_out/t_r4d.log
case $rc in 0|1) ;; *) echo "pytest rc=$rc: stopping"; exit $rc;; esac
Q="python -u tools/bench_qlora.py --steps 4 --warmup 2"
$T 200 $Q > gpurun_out/qlora_ab_default.json 2>&1 || exit 1
ILLM_GEMM_ENGINE=0 ILLM_LORA_ENGINE_NN=0 $T 200 $Q > gpurun_out/qlora_ab_noengine.json 2>&1 || exit 1
ILLM_GEMM_ENGINE=0 ILLM_LORA_ENGINE_NN=0 ILLM_TRAIN_ATTN=0 ILLM_TRAIN_CE=0 $T 200 $Q > gpurun_out/qlora_ab_r3path.json 2>&1 || exit 1
ILLM_TRAIN_ATTN=0 ILLM_TRAIN_CE=0 $T 200 $Q > gpurun_out/qlora_ab_engine_only.json 2>&1 || exit 1
for f in default noengine r3path engine_only; do echo $f; tail -1 gpurun_out/qlora_ab_$f.json | cut -c1-200; done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
$T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_qlora_r4 -o run --output-format csv -- python -u tools/bench_qlora.py --steps 2 --warmup 1 > gpurun_out/prof_qlora_r4.log 2>&1
echo "rocprof rc=$?"
