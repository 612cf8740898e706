#!/bin/bash
# Experiment: serial QP kernel at N=20 (LDS allows 8 instances per CU) for B = 256 .. 4096, i.e. one vs two
# waves per SIMD; and per-phase stamps at B = 1024 / 2048.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/occ
mkdir -p $O
cd $R
N=20 timeout -k 10 200 python3 tools/seg_sweep_b.py 256 512 1024 2048 4096 > $O/sweep_n20.txt 2>&1
cat $O/sweep_n20.txt
for b in 1024 2048; do B=$b N=20 timeout -k 10 120 python3 tools/qp_stamps.py > $O/stamps_n20_b$b.txt 2>&1; done
cat $O/stamps_n20_b*.txt
