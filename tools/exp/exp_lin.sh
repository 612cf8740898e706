#!/bin/bash
# linearize alone (tools/lin_probe.py) for the product library and diagnostic builds tools/_var/<v>.so
set -euo pipefail
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
for rep in 1 2; do
timeout -k 10 120 python3 tools/lin_probe.py
for v in "$@"; do echo "== $v"; SDFNMPC_LIB=$R/tools/_var/$v.so timeout -k 10 120 python3 tools/lin_probe.py; done
done
