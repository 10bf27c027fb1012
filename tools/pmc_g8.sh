#!/bin/bash
# PMC passes over the 8-phase GEMM, low-bit vs dense, one shape (GPU box):
# gpurun_out/pmc_g8_<impl>_{a,b,c}.csv + gpurun_out/pmc_g8_summary.txt
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p $R/gpurun_out; cd /tmp; export TMPDIR=/tmp
OP=${1:-gate_up}; M=${2:-8192}
for impl in g8 g8dense; do
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $R/gpurun_out/pmc8_a -o run -- python3 $R/tools/gemm_pmc.py $OP $M 10 $impl > $R/gpurun_out/pmc8_a.log 2>&1 || exit $?
  timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS --output-format csv -d $R/gpurun_out/pmc8_b -o run -- python3 $R/tools/gemm_pmc.py $OP $M 10 $impl > $R/gpurun_out/pmc8_b.log 2>&1 || exit $?
  timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $R/gpurun_out/pmc8_c -o run -- python3 $R/tools/gemm_pmc.py $OP $M 10 $impl > $R/gpurun_out/pmc8_c.log 2>&1 || exit $?
  for p in a b c; do f=$(find $R/gpurun_out/pmc8_$p -name "*counter_collection.csv" | head -1); cp "$f" $R/gpurun_out/pmc_g8_${impl}_$p.csv; done
  rm -rf $R/gpurun_out/pmc8_a $R/gpurun_out/pmc8_b $R/gpurun_out/pmc8_c
done
cd $R
python3 tools/pmc_summary.py gemm8p gpurun_out/pmc_g8_*_?.csv > gpurun_out/pmc_g8_summary.txt
cat gpurun_out/pmc_g8_summary.txt
