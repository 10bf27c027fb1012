#!/bin/bash
# round-4: token-axis LoRA reduction kernel numerics + QLoRA A/B (kernel vs library), same box
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T="timeout -k 10"
$T 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_train_kernels.py tests/test_gpu_training.py -m gpu > gpurun_out/t_r4v.log 2>&1
rc=$?; tail -3 gpurun_out/t_r4v.log; [ $rc -eq 0 ] || exit $rc
$T 300 python -u tools/bench_qlora.py --steps 8 --warmup 2 > gpurun_out/qlora_r4v_tn.json 2>&1 && \
ILLM_LORA_TN_KERNEL=0 $T 300 python -u tools/bench_qlora.py --steps 8 --warmup 2 > gpurun_out/qlora_r4v_lib.json 2>&1 && \
cd /tmp && export TMPDIR=/tmp && $T 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r4v -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_qlora.py --steps 3 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/prof_r4v.log 2>&1
rc=$?; cd $GRAFT_REPO_ROOT; for v in tn lib; do echo "$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/qlora_r4v_$v.json) $(grep -o '"value": [0-9.]*' gpurun_out/qlora_r4v_$v.json)"; done
f=$(ls gpurun_out/prof_r4v/*/run_kernel_stats.csv 2>/dev/null | head -1); [ -n "$f" ] && head -25 "$f" > gpurun_out/qlora_r4v_kstats.csv
find gpurun_out/prof_r4v -name '*.csv' ! -name '*stats*' -delete 2>/dev/null; exit $rc
