#!/bin/bash
# round-4: QLoRA default path (grouped LoRA, DMA attention, resident dense base) timing + rocprof; attention PMC
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T="timeout -k 10"
$T 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_training.py > gpurun_out/t_r4p.log 2>&1
rc=$?; tail -3 gpurun_out/t_r4p.log; [ $rc -eq 0 ] || exit $rc
$T 300 python -u tools/bench_qlora.py --steps 8 --warmup 2 > gpurun_out/qlora_r4p.json 2>&1
rc=$?; grep -h ms_per_step gpurun_out/qlora_r4p.json | cut -c1-400; [ $rc -eq 0 ] || exit $rc
bash tools/prof_qlora.sh && head -40 gpurun_out/prof_qlora_summary.txt
cd /tmp && export TMPDIR=/tmp
$T 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc_attn -o p1 -- python3 $GRAFT_REPO_ROOT/tools/attn_train_probe.py 512 > $GRAFT_REPO_ROOT/gpurun_out/pmc_attn.log 2>&1
rc=$?; cd $GRAFT_REPO_ROOT; echo "pmc rc=$rc"
python3 - <<'PY'
import csv, glob, collections
fs = glob.glob("gpurun_out/pmc_attn/**/*counter_collection.csv", recursive=True)
agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for f in fs:
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name", "")[:70]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        n[(k, r["Counter_Name"])] += 1
with open("gpurun_out/pmc_attn_summary.txt", "w") as o:
    for k, d in agg.items():
        o.write(k + "\n")
        for c, v in sorted(d.items()):
            o.write(f"   {c:28s} {v:.4g} (n={n[(k, c)]})\n")
print(open("gpurun_out/pmc_attn_summary.txt").read())
PY
rm -rf gpurun_out/pmc_attn
