#!/bin/bash
# A/B: the serial QP kernel with MFMA accumulators in AGPRs (product until round 4) vs in the unified VGPR
# file (-mllvm -amdgpu-mfma-vgpr-form), B = 1024 at N = 40 and 20, three runs each (HIP events)
set -euo pipefail
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/vf
mkdir -p $O
cd $R
for n in 40 20; do for rep in 1 2 3; do for drv in _plain _vf; do
  echo "N=$n drv$drv" >> $O/out.txt
  DRV=$drv B=1024 N=$n timeout -k 10 120 python3 tools/qp_stamps.py 2>&1 | grep kernel >> $O/out.txt
done; done; done
cat $O/out.txt
