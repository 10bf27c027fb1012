#!/bin/bash
# round-4: coalesced rank-update kernel numerics + QLoRA A/B; Infinity-Cache probe
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T="timeout -k 10"
$T 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_train_kernels.py -m gpu -k "lora_update or lora_tn" > gpurun_out/t_r4w.log 2>&1
rc=$?; tail -3 gpurun_out/t_r4w.log; [ $rc -eq 0 ] || exit $rc
$T 200 python -u tools/l3_probe.py > gpurun_out/l3_probe_b8.jsonl 2>&1 && \
PROBE_M=1 $T 200 python -u tools/l3_probe.py > gpurun_out/l3_probe_b1.jsonl 2>&1
rc=$?; cat gpurun_out/l3_probe_b8.jsonl gpurun_out/l3_probe_b1.jsonl | tail -12; [ $rc -eq 0 ] || exit $rc
$T 300 python -u tools/bench_qlora.py --steps 8 --warmup 2 > gpurun_out/qlora_r4w_rank.json 2>&1 && \
ILLM_LORA_RANK_KERNEL=0 $T 300 python -u tools/bench_qlora.py --steps 8 --warmup 2 > gpurun_out/qlora_r4w_addmm.json 2>&1
rc=$?; for v in rank addmm; do echo "$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/qlora_r4w_$v.json)"; done; exit $rc
