#!/bin/bash
# Serial QP kernel: the early window commit (each stage's hook commits the next position after its last window
# read) against the round-5 schedule (-DQP_LATE_COMMIT), plain timing drivers alternated, then the fine stamps
# (-DQP_STAMPS -DQP_FSTAMPS) of both.  Drivers: tools/_qp_stamps_drv_{hook,late,hookst,latest} (hipcc lines in
# DESIGN.md §3.4, the product's flags plus the defines).
set -euo pipefail
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R
for rep in 1 2 3; do
  for d in _hook _late; do echo "$d: $(DRV=$d timeout -k 10 120 python3 tools/qp_stamps.py 2>&1 | grep kernel)"; done
done
for d in _hookst _latest; do echo "== stamps $d"; DRV=$d timeout -k 10 120 python3 tools/qp_stamps.py 2>&1; done
