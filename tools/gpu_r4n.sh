#!/bin/bash
# round-4: smoke (fp32 torch reference), QLoRA default-path timing + kernel profile
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T="timeout -k 10"
$T 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r4n.txt 2>&1
rc=$?; tail -2 gpurun_out/smoke_r4n.txt; [ $rc -eq 0 ] || exit $rc
$T 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_families.py > gpurun_out/t_r4n.log 2>&1
rc=$?; tail -3 gpurun_out/t_r4n.log; [ $rc -eq 0 ] || exit $rc
$T 400 python -u tools/bench_qlora.py --steps 6 --warmup 2 > gpurun_out/qlora_r4n.json 2>&1
rc=$?; tail -2 gpurun_out/qlora_r4n.json; [ $rc -eq 0 ] || exit $rc
bash tools/prof_qlora.sh && head -45 gpurun_out/prof_qlora_summary.txt
