#!/bin/bash
# round-4: K-concatenated gate/up LoRA forward: parity test + same-box QLoRA A/B (alternated)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T="timeout -k 10"
$T 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_training.py tests/test_gpu_train_kernels.py -m gpu > gpurun_out/t_r4ac.log 2>&1
rc=$?; tail -3 gpurun_out/t_r4ac.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  $T 300 python -u tools/bench_qlora.py --steps 8 --warmup 2 > gpurun_out/qlora_ab_rows_$i.json 2>&1 || exit $?
  ILLM_LORA_KCAT_ROWS=0 $T 300 python -u tools/bench_qlora.py --steps 8 --warmup 2 > gpurun_out/qlora_ab_norows_$i.json 2>&1 || exit $?
done
for f in gpurun_out/qlora_ab_*rows*.json; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' $f) $(grep -o '"loss[a-z_]*": [^,]*' $f | head -2 | tr '\n' ' ')"; done
