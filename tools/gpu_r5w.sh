#!/bin/bash
# round 5: dense 8-phase GEMM with 3 weight buffers (_C.so) vs 2 (_C_b2.so): tests, bf16 + fp8 sweeps, prefill
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_gemm8p.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5w_pytest.log 2>&1 || { tail -30 gpurun_out/r5w_pytest.log; exit 2; }
tail -2 gpurun_out/r5w_pytest.log
: > gpurun_out/r5w_g8.jsonl
for lib in _C.so _C_b2.so; do
  echo "# $lib" >> gpurun_out/r5w_g8.jsonl
  IPEX_LLM_AMD_LIB=$lib timeout -k 10 300 python tools/bench_g8.py sym_int4 --m 8192,1024 --dense >> gpurun_out/r5w_g8.jsonl || exit 3
done
: > gpurun_out/r5w_fp8.jsonl
for lib in _C.so _C_b2.so; do
  echo "# $lib" >> gpurun_out/r5w_fp8.jsonl
  IPEX_LLM_AMD_LIB=$lib timeout -k 10 300 python tools/fp8_gemm_bench.py >> gpurun_out/r5w_fp8.jsonl || exit 4
done
for lib in _C.so _C_b2.so; do
  IPEX_LLM_AMD_LIB=$lib BENCH_BATCH=8 timeout -k 10 200 python bench.py --steps 16 --warmup 4 --no-tp-side > gpurun_out/r5w_b8_$lib.log 2>&1 || { tail -5 gpurun_out/r5w_b8_$lib.log; exit 5; }
  echo "$lib $(tail -1 gpurun_out/r5w_b8_$lib.log | grep -o '"first_token_latency_ms": [0-9.]*')"
done
