#!/bin/bash
# Experiment: the segmented QP kernel under the max-ilp scheduling strategy (_build/allilp) vs the product
set -euo pipefail
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R
for lib in product allilp product allilp; do
  L=$R/sdf-nmpc_amd/lib/libsdfnmpc.so; [ $lib = allilp ] && L=$R/_build/allilp/libsdfnmpc.so
  echo "== $lib N=60: $(SDFNMPC_LIB=$L N=60 timeout -k 10 120 python3 tools/seg_sweep_b.py 1 512 2>&1 | grep B= | tr '\n' ' ')"
done
