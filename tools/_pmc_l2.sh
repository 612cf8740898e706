#!/bin/bash
# L2-side counters of the preparation kernels (sdf_mlp's weight re-streaming): one rocprofv3 pass per set.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out/pmcl2; mkdir -p $O
timeout -s KILL 60 rocprofv3 --list-avail > $O/avail.txt 2>&1 || true
grep -oE "(TCP|TCC)_[A-Z0-9_]+" $O/avail.txt | sort -u > $O/tc_names.txt || true
n=0
for set in "TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum" "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" "FETCH_SIZE" "SQ_INSTS_VMEM_RD SQ_INSTS_MFMA SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES"; do
  n=$((n+1))
  for tile in 32 64; do
    TILE=$tile timeout -s KILL 90 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $O/p${n}_t$tile -o p -- python3 $R/tools/sdf_prep_drv.py > /dev/null 2>> $O/err.log || echo "pass $n tile $tile failed" >> $O/err.log
  done
done
echo done
