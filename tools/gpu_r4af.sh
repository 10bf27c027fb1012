#!/bin/bash
# round-4: dense GLU (shared conversions, 2-deep loads): tests + verify-row A/B (max rows 16 vs 2), same box
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T="timeout -k 10"
$T 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -m gpu -k dense_glu > gpurun_out/t_r4af.log 2>&1
rc=$?; tail -2 gpurun_out/t_r4af.log; [ $rc -eq 0 ] || exit $rc
ILLM_DENSE_GLU_MAX_M=16 $T 300 python -u tools/spec_bench.py --ks 2,3 > gpurun_out/spec_glu16_r4.jsonl 2>&1 || exit $?
$T 300 python -u tools/spec_bench.py --ks 2,3 > gpurun_out/spec_glu2_r4.jsonl 2>&1 || exit $?
for f in spec_glu16_r4 spec_glu2_r4; do echo $f; grep -o '"mode": "[a-z_0-9]*"[^}]*"ms_per_token": [0-9.]*\|"k": [0-9]*\|"generated_token_agreement": [0-9.]*' gpurun_out/$f.jsonl | tr '\n' ' '; echo; done
