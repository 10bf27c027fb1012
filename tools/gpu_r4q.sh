#!/bin/bash
# round-4: PMC of the B=8 decode step's kernels (attention split + combine, GEMVs)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T="timeout -k 10"
cd /tmp && export TMPDIR=/tmp
$T 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc_dec -o p1 -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/pmc_dec.log 2>&1
rc=$?; cd $GRAFT_REPO_ROOT; echo "pmc rc=$rc"
$T 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum GRBM_GUI_ACTIVE --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc_dec2 -o p2 -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/pmc_dec2.log 2>&1
echo "pmc2 rc=$?"
python3 - <<'PY'
import csv, glob, collections
out = open("gpurun_out/pmc_dec_summary.txt", "w")
for d in ("pmc_dec", "pmc_dec2"):
    fs = glob.glob(f"gpurun_out/{d}/**/*counter_collection.csv", recursive=True)
    agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
    for f in fs:
        for r in csv.DictReader(open(f)):
            k = r.get("Kernel_Name", "")[:90]
            if not any(s in k for s in ("attn", "gemv", "norm", "combine")):
                continue
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            n[(k, r["Counter_Name"])] += 1
    for k, dd in agg.items():
        out.write(k + "\n")
        for c, v in sorted(dd.items()):
            out.write(f"   {c:28s} {v:.4g} (n={n[(k, c)]})\n")
out.close()
print(open("gpurun_out/pmc_dec_summary.txt").read()[:6000])
PY
rm -rf gpurun_out/pmc_dec gpurun_out/pmc_dec2
