#!/bin/bash
# The C3 preparation phase (tools/sdf_bench.py: sdf_hoist + sdf_mlp beside linearize): product vs diagnostic builds
set -euo pipefail
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/prep; mkdir -p $O
cd $R
for rep in 1 2; do
timeout -k 10 120 python3 tools/sdf_bench.py > $O/product_$rep.txt 2>&1
for v in "$@"; do SDFNMPC_LIB=$R/_build/$v/libsdfnmpc.so timeout -k 10 120 python3 tools/sdf_bench.py > $O/${v}_$rep.txt 2>&1; done
done
grep -H "ms/prep" $O/*.txt
