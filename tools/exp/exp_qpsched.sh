#!/bin/bash
# Experiment: the serial QP kernel under LLVM's alternative AMDGPU scheduling strategies (driver builds)
set -euo pipefail
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R
for d in ${DRVS:-_vf _max-ilp _max-memory-clause _iterative-ilp}; do
  echo "$d: $(DRV=$d B=1024 N=40 timeout -k 10 120 python3 tools/qp_stamps.py 2>&1 | grep kernel)"
done
