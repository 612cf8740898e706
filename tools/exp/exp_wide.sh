#!/bin/bash
# The C5 wide-net preparation phase: the product build against diagnostic builds (tools/build_variant.sh)
set -euo pipefail
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/wide; mkdir -p $O
cd $R
timeout -k 10 120 python3 tools/wide_bench.py > $O/product.txt 2>&1
for v in "$@"; do SDFNMPC_LIB=$R/_build/$v/libsdfnmpc.so timeout -k 10 120 python3 tools/wide_bench.py > $O/$v.txt 2>&1; done
grep -H "ms/prep\|sdf_wide_gemm" $O/*.txt
