#!/bin/bash
# PMC counter passes over the prefill low-bit GEMM (GPU box), counters only
# (no trace domains): gpurun_out/pmc_gemm_{a,b,c}.csv
set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd /tmp; export TMPDIR=/tmp
OP=${1:-gate_up}; M=${2:-1024}
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $R/gpurun_out/pmcg_a -o run -- python3 $R/tools/gemm_pmc.py $OP $M 20 > $R/gpurun_out/pmcg_a.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS --output-format csv -d $R/gpurun_out/pmcg_b -o run -- python3 $R/tools/gemm_pmc.py $OP $M 20 > $R/gpurun_out/pmcg_b.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $R/gpurun_out/pmcg_c -o run -- python3 $R/tools/gemm_pmc.py $OP $M 20 > $R/gpurun_out/pmcg_c.log 2>&1 || exit $?
cd $R
for p in a b c; do f=$(find gpurun_out/pmcg_$p -name "*counter_collection.csv" | head -1); cp "$f" gpurun_out/pmc_gemm_$p.csv; done
rm -rf gpurun_out/pmcg_a gpurun_out/pmcg_b gpurun_out/pmcg_c
