#!/bin/bash
# round 5: GEMM out/accumulate + transposed skinny GEMM tests, training tests, QLoRA step (+ rocprof), full GPU suite
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm8p.py tests/test_gpu_dense_gemv.py tests/test_gpu_training.py tests/test_gpu_train_kernels.py -q -x --timeout 200 --timeout-method thread > gpurun_out/r5m_tests.log 2>&1 || { tail -40 gpurun_out/r5m_tests.log; exit 2; }
tail -1 gpurun_out/r5m_tests.log
timeout -k 10 400 python -u tools/bench_qlora.py --steps 6 --warmup 2 > gpurun_out/r5m_qlora.log 2>&1 || { tail -20 gpurun_out/r5m_qlora.log; exit 5; }
tail -1 gpurun_out/r5m_qlora.log | cut -c1-400
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d "$R/gpurun_out/prof_ql" -o run -- python3 "$R/tools/bench_qlora.py" --steps 3 --warmup 1 > "$R/gpurun_out/r5m_ql.log" 2>&1 || exit 6
cd "$R"
db=$(find gpurun_out/prof_ql -name "*.db" | head -1)
python3 tools/prof_summary.py "$db" 40 > gpurun_out/r5m_ql_summary.txt 2>&1
echo "Cijk kernels: $(grep -c Cijk gpurun_out/r5m_ql_summary.txt)"
rm -rf gpurun_out/prof_ql
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 280 --timeout-method thread > gpurun_out/r5m_pytest.log 2>&1
rc=$?
tail -6 gpurun_out/r5m_pytest.log
exit $rc
