#!/bin/bash
# linearize alone (tools/lin_probe.py): SQ counters of the kernel (one rocprofv3 --pmc pass each)
set -euo pipefail
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/pmc_lin; mkdir -p $O
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $O/a -o p -- python3 $R/tools/lin_probe.py > $O/a.txt 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_WR SQ_INSTS_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_VMEM_RD --kernel-trace --output-format csv -d $O/b -o p -- python3 $R/tools/lin_probe.py > $O/b.txt 2>&1
python3 $R/tools/pmc_kernel_mean.py linearize_kernel $O/a $O/b
