#!/bin/bash
# QP per-phase cycles vs batch size (shared-CU / memory pressure diagnostic) and driver variants
set -euo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
for b in ${BS:-1024 256 64}; do
  echo "#### B=$b"
  B=$b timeout -k 10 200 python tools/qp_stamps.py
  for d in ${VARS:-}; do echo "-- $d"; timeout -k 10 60 tools/_qp_stamps_drv_$d /tmp/qp_in.bin; done
done
