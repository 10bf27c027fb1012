#!/bin/bash
# round 5: dense 8-phase memory probe, speculative bench (MFMA dense verify), full GPU suite
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 200 python -u tools/g8_probe.py > gpurun_out/r5i_probe.jsonl 2> gpurun_out/r5i_probe.err || exit 3
grep -v amdgpu gpurun_out/r5i_probe.jsonl
timeout -k 10 420 python -u tools/spec_bench.py --ks 1,2,3 --new 128 > gpurun_out/r5i_spec.jsonl 2> gpurun_out/r5i_spec.err || exit 4
grep -v amdgpu gpurun_out/r5i_spec.jsonl | cut -c1-300
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 280 --timeout-method thread > gpurun_out/r5i_pytest.log 2>&1
rc=$?
tail -8 gpurun_out/r5i_pytest.log
exit $rc
