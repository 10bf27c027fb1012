#!/bin/bash
# round-4: dense GLU decode kernel: tests + bf16-target / speculative A/B (same box)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T="timeout -k 10"
$T 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_speculative.py tests/test_gpu_families.py -m gpu > gpurun_out/t_r4ae.log 2>&1
rc=$?; tail -3 gpurun_out/t_r4ae.log; [ $rc -eq 0 ] || exit $rc
$T 300 python -u tools/spec_bench.py --ks 2,3 > gpurun_out/spec_glu_r4.jsonl 2>&1 || exit $?
ILLM_DENSE_GLU=0 $T 300 python -u tools/spec_bench.py --ks 2,3 > gpurun_out/spec_noglu_r4.jsonl 2>&1 || exit $?
for f in spec_glu_r4 spec_noglu_r4; do echo $f; grep -o '"mode": "[a-z_0-9]*"[^}]*"ms_per_token": [0-9.]*\|"k": [0-9]*\|"speedup_vs_bf16": [0-9.]*\|"generated_token_agreement": [0-9.]*' gpurun_out/$f.jsonl | tr '\n' ' '; echo; done
