#!/bin/bash
# QLoRA whole-step hipGraph with the round-3 training kernels (LoRA node, RMSNorm/RoPE/act*up fwd+bwd)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python tools/bench_qlora.py --graph --steps 8 --warmup 2 > gpurun_out/qlora_graph_r3.log 2>&1 || { tail -20 gpurun_out/qlora_graph_r3.log; exit 1; }
tail -1 gpurun_out/qlora_graph_r3.log | grep -o '"ms_per_step": [0-9.]*\|"loss_last": [0-9.]*\|"loss_first": [0-9.]*' | tr '\n' ' '
