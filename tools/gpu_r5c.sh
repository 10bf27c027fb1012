#!/bin/bash
# round 5: full GPU suite + decode traces (B=1, B=8) on the v3 attention defaults
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 280 --timeout-method thread > gpurun_out/r5c_pytest.log 2>&1
rc=$?
tail -5 gpurun_out/r5c_pytest.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
bash tools/prof_decode.sh || exit $?
head -14 gpurun_out/prof_b1_summary.txt; head -16 gpurun_out/prof_b8_summary.txt
exit $rc
