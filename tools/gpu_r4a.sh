#!/bin/bash
# round-4 GPU step: MFMA GEMM engine tests + Llama-3-8B shape sweep
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_mfgemm.py > gpurun_out/t_mfgemm.log 2>&1; echo rc=$? >> gpurun_out/t_mfgemm.log; tail -5 gpurun_out/t_mfgemm.log; grep -q "rc=0" gpurun_out/t_mfgemm.log && GEMM_M=1024,4096 timeout -k 10 300 python -u tools/bench_mfgemm.py > gpurun_out/mfg_sweep1.jsonl 2>&1; cat gpurun_out/mfg_sweep1.jsonl | tail -20
