set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python tools/bench_kernels.py --only gemv > gpurun_out/bk_gemv.log 2>&1 &&
BENCH_BATCH=1 timeout -k 10 300 python bench.py --steps 64 --warmup 8 > gpurun_out/bench_b1.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 64 --warmup 8 > gpurun_out/bench_b8.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu.log; tail -2 gpurun_out/bench_b1.log gpurun_out/bench_b8.log
exit $rc
