#!/bin/bash
# round 6 final tree: full GPU suite, smoke, bench B=1 / B=8 (two runs each), decode traces
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6m_pytest.log 2>&1 || { tail -40 gpurun_out/r6m_pytest.log; exit 2; }
tail -3 gpurun_out/r6m_pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6m_smoke.log 2>&1 || { tail -20 gpurun_out/r6m_smoke.log; exit 3; }
tail -2 gpurun_out/r6m_smoke.log
: > gpurun_out/r6m_bench.jsonl
for i in 1 2; do for B in 8 1; do
  BENCH_BATCH=$B timeout -k 10 300 python bench.py > gpurun_out/r6m_tmp.log 2>&1 || { tail -5 gpurun_out/r6m_tmp.log; exit 4; }
  tail -1 gpurun_out/r6m_tmp.log | tee -a gpurun_out/r6m_bench.jsonl
done; done
