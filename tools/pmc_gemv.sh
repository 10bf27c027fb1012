set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd /tmp; export TMPDIR=/tmp
timeout -k 10 120 $R/tools/probe/stream_probe > $R/gpurun_out/stream_probe.log 2>&1 || exit $?
for op in glu down; do
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace --stats -d $R/gpurun_out/pmc_${op}_a -o run -- python3 $R/tools/gemv_pmc.py $op 1 40 > $R/gpurun_out/pmc_${op}_a.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace -d $R/gpurun_out/pmc_${op}_b -o run -- python3 $R/tools/gemv_pmc.py $op 1 40 > $R/gpurun_out/pmc_${op}_b.log 2>&1 || exit $?
done
cd $R; find gpurun_out/pmc_* -name "*counter_collection.csv" | head; 
