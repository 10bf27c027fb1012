#!/bin/bash
# round 5: 8-phase GEMM PMC (low-bit vs dense), speculative round trace,
# GPU suite with the per-test kernel-error check
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 180 python -u -m pytest tests/test_gpu_gemm8p.py tests/test_gpu_kernels.py tests/test_gpu_training.py -k 'gemm or dequantize_device or lora or qlora' -q -x --timeout 100 --timeout-method thread > gpurun_out/r5g_g8tests.log 2>&1 || { tail -30 gpurun_out/r5g_g8tests.log; exit 2; }
tail -2 gpurun_out/r5g_g8tests.log
timeout -k 10 300 python -u tools/bench_g8.py sym_int4 --m 8192,1024 --dense > gpurun_out/r5g_g8d.jsonl 2> gpurun_out/r5g_g8d.err || exit 3
echo "g8d bench ok"
ILLM_G8_DSCHED=3 timeout -k 10 300 python -u tools/bench_g8.py sym_int4 --m 8192,1024 --dense > gpurun_out/r5g_g8d_ds3.jsonl 2> gpurun_out/r5g_g8d_ds3.err || exit 3
echo "g8d dsched3 bench ok"
bash tools/pmc_g8.sh gate_up 8192 > gpurun_out/r5g_pmc.log 2>&1 || { tail -20 gpurun_out/r5g_pmc.log; exit 3; }
echo "pmc ok"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d "$R/gpurun_out/spec_prof" -o run -- python3 "$R/tools/spec_bench.py" --ks 2 --new 64 --skip-plain > "$R/gpurun_out/r5g_spec.log" 2>&1 || exit 4
cd "$R"
db=$(find gpurun_out/spec_prof -name "*.db" | head -1)
python3 tools/prof_by_grid.py "$db" 45 --after attn_prefill > gpurun_out/r5g_spec_by_grid.txt 2>&1
rm -rf gpurun_out/spec_prof
head -30 gpurun_out/r5g_spec_by_grid.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 280 --timeout-method thread > gpurun_out/r5g_pytest.log 2>&1
rc=$?
tail -12 gpurun_out/r5g_pytest.log
exit $rc
