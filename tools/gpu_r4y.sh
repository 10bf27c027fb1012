#!/bin/bash
# round-4: dense prefill shadow test + TTFT; lora_tn split-policy sweep
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T="timeout -k 10"
$T 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_model.py tests/test_gpu_encoders.py -m gpu -k "dense_shadow or multimodal" > gpurun_out/t_r4y.log 2>&1
rc=$?; tail -3 gpurun_out/t_r4y.log; [ $rc -eq 0 ] || exit $rc
for rw in "128 2048" "256 1024" "512 1024" "256 2048"; do
  set -- $rw
  ILLM_LORA_TN_ROWS=$1 ILLM_LORA_TN_WGS=$2 $T 120 python -u tools/bench_lora_tn.py >> gpurun_out/lora_tn_sweep_r4.jsonl 2>&1 || exit $?
done
cat gpurun_out/lora_tn_sweep_r4.jsonl | grep sum_
$T 300 python -u bench.py --batch 1 --steps 64 --warmup 8 > gpurun_out/bench_b1_r4y.json 2>&1 && \
$T 300 python -u bench.py --steps 64 --warmup 8 > gpurun_out/bench_b8_r4y.json 2>&1
rc=$?; for b in 1 8; do tail -1 gpurun_out/bench_b${b}_r4y.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print($b, d['value'], d['ms_per_step'], d['first_token_latency_ms'], d['config'].get('prefill_dense_shadow_gb'))"; done; exit $rc
