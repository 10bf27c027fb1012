#!/bin/bash
# round-3: new GPU tests (peer all-reduce f32/two-shot, TP graph decode, grouped MoE GEMM), then
# the o_proj-combine A/B at B=1 and Mixtral first-token latency
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_allreduce.py tests/test_gpu_tp.py tests/test_gpu_moe_gemm.py tests/test_gpu_moe.py -x -v --timeout 200 --timeout-method thread > gpurun_out/pt_r3b.log 2>&1
rc=$?
tail -4 gpurun_out/pt_r3b.log
[ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ] && exit $rc
for cfg in "ILLM_OPROJ_COMBINE=0" "ILLM_OPROJ_COMBINE=1 ILLM_OPROJ_KS=32 ILLM_OPROJ_NW=8" "ILLM_OPROJ_COMBINE=1 ILLM_OPROJ_KS=16 ILLM_OPROJ_NW=8" "ILLM_OPROJ_COMBINE=1 ILLM_OPROJ_KS=32 ILLM_OPROJ_NW=4" "ILLM_OPROJ_COMBINE=0"; do
  env $cfg BENCH_BATCH=1 timeout -k 10 200 python bench.py --steps 128 --warmup 8 > gpurun_out/b1_cfg.log 2>&1 || exit $?
  echo "$cfg $(tail -1 gpurun_out/b1_cfg.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["first_token_latency_ms"], d["sample_next_ids"])')"
done
BENCH_BATCH=1 timeout -k 10 300 python bench.py --model mixtral-8x7b --steps 32 --warmup 4 > gpurun_out/mixtral_b1.log 2>&1 || exit $?
tail -1 gpurun_out/mixtral_b1.log | cut -c1-400
