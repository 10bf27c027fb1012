#!/bin/bash
# round-4: strict speculative agreement tests + spec bench with the GLU row cap at 16
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T="timeout -k 10"
$T 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_speculative.py tests/test_gpu_kernels.py -m gpu -k "speculative or dense" > gpurun_out/t_r4ag.log 2>&1
rc=$?; tail -3 gpurun_out/t_r4ag.log; [ $rc -eq 0 ] || exit $rc
$T 300 python -u tools/spec_bench.py --ks 2,4,6 > gpurun_out/spec_final_r4.jsonl 2>&1 || exit $?
grep -o '"mode": "[a-z_0-9]*"[^}]*"ms_per_token": [0-9.]*\|"k": [0-9]*\|"speedup_vs_bf16": [0-9.]*\|"generated_token_agreement": [0-9.]*' gpurun_out/spec_final_r4.jsonl | tr '\n' ' '
