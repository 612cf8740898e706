#!/bin/bash
# sdf_mlp diagnostic variants (tools/build_variant.sh builds under _build/<name>/); SERIAL=1: linearize
# after the SDF kernel on the same stream, so the SDF kernel's time is its own
set -euo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
export SDFNMPC_SERIAL_PREP=${SERIAL:-0}
timeout -k 10 120 python tools/sdf_bench.py
for v in ${VARS:-}; do SDFNMPC_LIB=$R/_build/$v/libsdfnmpc.so timeout -k 10 120 python tools/sdf_bench.py; done
