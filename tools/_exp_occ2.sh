#!/bin/bash
# Experiment: the serial QP kernel at two waves per SIMD (register allocation capped at 256, QP_LB_WAVES=2)
# vs the product allocation (375 registers, one wave per SIMD), N = 20 (LDS admits 7 instances per CU).
set -euo pipefail
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/occ2
mkdir -p $O
cd $R
for drv in _plain _lb2; do for b in 1024 2048 4096; do
  echo "drv$drv B=$b" >> $O/out.txt
  DRV=$drv B=$b N=20 timeout -k 10 120 python3 tools/qp_stamps.py 2>&1 | grep kernel >> $O/out.txt
done; done
cat $O/out.txt
