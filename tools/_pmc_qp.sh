set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 200 python $R/tools/qp_stamps.py > $R/gpurun_out/st.log 2>&1
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" "SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_INSTS_BRANCH"; do
  n=$((n+1))
  timeout -k 10 120 rocprofv3 --pmc $set --kernel-trace -d $R/gpurun_out/pmc$n -o p -- $R/tools/_qp_stamps_drv /tmp/qp_in.bin >> $R/gpurun_out/st.log 2>&1
done
