#!/bin/bash
# Experiment: the serial QP kernel's record-stream prefetch depth (QP_RING_DEPTH 3 / 4 / 5) at B = 256 and
# 1024; N = 39 keeps four instances per CU at every depth (N = 40 at depth 4 needs 64 B more LDS).
set -euo pipefail
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/ring; mkdir -p $O; : > $O/out.txt
cd $R
for n in 39 40; do for b in 256 1024; do for d in 3 4 5; do
  echo "N=$n B=$b depth $d: $(DRV=_pd$d B=$b N=$n timeout -k 10 120 python3 tools/qp_stamps.py 2>&1 | grep kernel)" >> $O/out.txt
done; done; done
cat $O/out.txt
