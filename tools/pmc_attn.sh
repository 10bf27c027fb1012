#!/bin/bash
# PMC counter passes over the prefill flash attention (GPU box), counters only:
# gpurun_out/pmc_attn_{a,b,c}.csv
set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd /tmp; export TMPDIR=/tmp
T=${1:-4096}
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $R/gpurun_out/pmca_a -o run -- python3 $R/tools/attn_pmc.py $T 10 > $R/gpurun_out/pmca_a.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS --output-format csv -d $R/gpurun_out/pmca_b -o run -- python3 $R/tools/attn_pmc.py $T 10 > $R/gpurun_out/pmca_b.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $R/gpurun_out/pmca_c -o run -- python3 $R/tools/attn_pmc.py $T 10 > $R/gpurun_out/pmca_c.log 2>&1 || exit $?
cd $R
for p in a b c; do f=$(find gpurun_out/pmca_$p -name "*counter_collection.csv" | head -1); cp "$f" gpurun_out/pmc_attn_$p.csv; done
rm -rf gpurun_out/pmca_a gpurun_out/pmca_b gpurun_out/pmca_c
python3 - <<'PY'
import csv, collections
agg = collections.defaultdict(float)
for p in "abc":
    for r in csv.DictReader(open(f"gpurun_out/pmc_attn_{p}.csv")):
        if "attn_prefill" in r["Kernel_Name"]:
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
            agg["VGPR"] = float(r["VGPR_Count"]); agg["AGPR"] = float(r.get("Accum_VGPR_Count") or 0)
for k, v in sorted(agg.items()):
    print(f"{k:28s} {v:.4g}")
PY
