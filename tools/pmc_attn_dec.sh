#!/bin/bash
# kernel trace + PMC passes over the decode attention (GPU box):
#   tools/pmc_attn_dec.sh B L rope  -> gpurun_out/pmc_attn_dec_B<B>_<rope>.txt
set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd /tmp; export TMPDIR=/tmp
B=${1:-1}; L=${2:-1024}; RP=${3:-1}; TAG=B${B}_r${RP}
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pad_t -o run -- python3 $R/tools/attn_dec_pmc.py $B $L 20 $RP > $R/gpurun_out/pad_t.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $R/gpurun_out/pad_a -o run -- python3 $R/tools/attn_dec_pmc.py $B $L 20 $RP > $R/gpurun_out/pad_a.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS --output-format csv -d $R/gpurun_out/pad_b -o run -- python3 $R/tools/attn_dec_pmc.py $B $L 20 $RP > $R/gpurun_out/pad_b.log 2>&1 || exit $?
cd $R
python3 - "$TAG" <<'PY'
import csv, collections, glob, sys
tag = sys.argv[1]
out = open(f"gpurun_out/pmc_attn_dec_{tag}.txt", "w")
st = glob.glob("gpurun_out/pad_t/**/*kernel_stats.csv", recursive=True)
for r in csv.DictReader(open(st[0])):
    out.write(f"{r['Name'][:90]:92s} calls {r['Calls']:>5s} avg_us {float(r['AverageNs'])/1e3:8.2f}\n")
for p in "ab":
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(f"gpurun_out/pad_{p}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"][:60]
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            agg[k]["VGPR"] = float(r["VGPR_Count"])
    for k, d in agg.items():
        out.write(f"-- {k}\n")
        for c, v in sorted(d.items()):
            out.write(f"   {c:26s} {v:.4g}\n")
out.close()
print(open(f"gpurun_out/pmc_attn_dec_{tag}.txt").read())
PY
rm -rf gpurun_out/pad_t gpurun_out/pad_a gpurun_out/pad_b
