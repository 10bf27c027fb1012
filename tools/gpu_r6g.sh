#!/bin/bash
# round 6: register-staged early x (XM 1 / 2 instantiations): numerics at the real
# shapes, production-shape parity, A/B vs _C_noearly.so, stamps, decode traces
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 200 python -u tools/debug_glu.py 2>&1 | grep -v amdgpu.ids
timeout -k 10 700 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_prodshape.py tests/test_gpu_model.py -x -q --timeout 300 --timeout-method thread -k "gemv or norm or glu or decode or argmax or llama3 or graph" > gpurun_out/r6g_pytest.log 2>&1 || { tail -40 gpurun_out/r6g_pytest.log; exit 2; }
tail -2 gpurun_out/r6g_pytest.log
: > gpurun_out/r6g_ab.jsonl
run() {  # B, lib
  IPEX_LLM_AMD_LIB=$2 BENCH_BATCH=$1 timeout -k 10 200 python bench.py --steps 128 --warmup 8 --no-tp-side > gpurun_out/r6g_tmp.log 2>&1 || { tail -5 gpurun_out/r6g_tmp.log; return 1; }
  tail -1 gpurun_out/r6g_tmp.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(json.dumps({'B': $1, 'lib': '$2', 'tok_s': d['value'], 'ms': d['ms_per_step'], 'ftl': d['first_token_latency_ms']}))" | tee -a gpurun_out/r6g_ab.jsonl
}
for i in 1 2; do
  for lib in _C.so _C_noearly.so; do run 8 $lib || exit 3; run 1 $lib || exit 3; done
done
PROBE_MODE=s timeout -k 10 120 tools/probe/gemv5_stamps_xr > gpurun_out/r6g_stamps.jsonl 2>&1 || { tail -5 gpurun_out/r6g_stamps.jsonl; exit 7; }
grep timeline gpurun_out/r6g_stamps.jsonl
for B in 8 1; do
BENCH_BATCH=$B timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/prof_b$B" -o run -- python3 "$R/bench.py" --steps 32 --warmup 4 --no-tp-side > "$R/gpurun_out/r6g_prof$B.log" 2>&1 || exit 5
db=$(find gpurun_out/prof_b$B -name "*.db" | head -1)
python3 tools/decode_trace_summary.py "$db" 5 > gpurun_out/r6g_trace_b$B.txt 2>&1 || exit 6
rm -rf gpurun_out/prof_b$B
head -10 gpurun_out/r6g_trace_b$B.txt
done
