#!/bin/bash
# Experiment: sdf_mlp time against the row count at N = 40 (32-row tiles, 512 workgroup slots): B = 799
# is 2.0 rounds of tiles, 1024 is 2.56 (the C3 batch), 1199 is 3.0; the preparation phase and its kernels.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/sdfq; mkdir -p $O; : > $O/out.txt
for b in 400 600 799 900 1024 1100 1199 1400 1598; do
  timeout -k 10 120 python3 $R/tools/sdf_bench.py $b 40 32 >> $O/out.txt 2>&1
done
cat $O/out.txt
