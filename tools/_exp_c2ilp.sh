#!/bin/bash
# Experiment: the C2 per-call path (resident SDF server) built with max-ilp (_build/allilp) vs the product
set -euo pipefail
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R
for lib in product allilp product allilp; do
  L=$R/sdf-nmpc_amd/lib/libsdfnmpc.so; [ $lib = allilp ] && L=$R/_build/allilp/libsdfnmpc.so
  echo "== $lib"; SDFNMPC_LIB=$L timeout -k 10 120 python3 tools/c2_probe.py 2>&1 | grep -v amdgpu.ids
done
