#!/bin/bash
# GEMV breakdown probes (ablation builds), capturable AdamW test, QLoRA graph vs eager
set -o pipefail
mkdir -p gpurun_out
for a in 0 1 2 3 4 7; do
  timeout -k 10 120 tools/probe/gemv5_probe_a$a >> gpurun_out/gemv5_probe.jsonl 2>&1 || exit $?
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_training.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pt_train.log 2>&1
rc=$?; tail -3 gpurun_out/pt_train.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python tools/bench_qlora.py --steps 6 --warmup 2 --graph > gpurun_out/qlora_graph.log 2>&1 || exit $?
tail -1 gpurun_out/qlora_graph.log | cut -c1-300
timeout -k 10 400 python tools/bench_qlora.py --steps 6 --warmup 2 > gpurun_out/qlora_eager.log 2>&1 || exit $?
tail -1 gpurun_out/qlora_eager.log | cut -c1-300
