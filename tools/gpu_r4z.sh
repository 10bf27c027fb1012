#!/bin/bash
# round-4: LoRA gradient slab (one fill + one cast per node) tests + QLoRA bench
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T="timeout -k 10"
$T 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_train_kernels.py tests/test_gpu_training.py -m gpu > gpurun_out/t_r4z.log 2>&1
rc=$?; tail -3 gpurun_out/t_r4z.log; [ $rc -eq 0 ] || exit $rc
$T 300 python -u tools/bench_qlora.py --steps 8 --warmup 2 > gpurun_out/qlora_r4z.json 2>&1 && \
ILLM_LORA_TN_KERNEL=0 $T 300 python -u tools/bench_qlora.py --steps 8 --warmup 2 > gpurun_out/qlora_r4z_lib.json 2>&1
rc=$?; for v in r4z r4z_lib; do echo "$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/qlora_$v.json) $(grep -o '"value": [0-9.]*' gpurun_out/qlora_$v.json)"; done; exit $rc
