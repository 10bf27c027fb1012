#!/bin/bash
# GPU box: attention tests + long-context decode bench + 32K profile
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "attn or decode or combine or rwkv" > gpurun_out/pytest_attn.log 2>&1 || { tail -30 gpurun_out/pytest_attn.log; exit 1; }
tail -2 gpurun_out/pytest_attn.log
PLENS="1024 8192 32768" bash tools/gpu_longctx.sh 2>&1 | grep "^P=" || exit 1
bash tools/prof_longctx.sh 32768
