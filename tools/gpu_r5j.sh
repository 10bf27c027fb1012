#!/bin/bash
# round 5: 8-phase rasterization-group sweep (ILLM_G8_GM), dense MFMA GEMV tests + spec bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
for gm in 4 8 16 32; do
  ILLM_G8_GM=$gm timeout -k 10 200 python -u tools/g8_probe.py --shapes > gpurun_out/r5j_gm$gm.jsonl 2> gpurun_out/r5j_gm$gm.err || exit 3
  echo "gm $gm: $(grep -v amdgpu gpurun_out/r5j_gm$gm.jsonl | python3 -c 'import sys,json; print([ (d["M"], d["op"], d["vs_lib"]) for d in map(json.loads, sys.stdin)])')"
done
timeout -k 10 200 python -u -m pytest tests/test_gpu_dense_gemv.py tests/test_gpu_kernels.py -k "dense" -q -x --timeout 100 --timeout-method thread > gpurun_out/r5j_tests.log 2>&1 || { tail -30 gpurun_out/r5j_tests.log; exit 2; }
tail -1 gpurun_out/r5j_tests.log
timeout -k 10 420 python -u tools/spec_bench.py --ks 1,3 --new 128 > gpurun_out/r5j_spec.jsonl 2> gpurun_out/r5j_spec.err || exit 4
grep -v amdgpu gpurun_out/r5j_spec.jsonl | cut -c1-300
