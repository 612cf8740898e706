#!/bin/bash
# VAE stem: the product build against diagnostic builds (tools/build_variant.sh) at B = 512
set -euo pipefail
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/stem
mkdir -p $O
cd $R
timeout -k 10 120 python3 tools/vae_bench.py > $O/product.txt 2>&1
for v in "$@"; do SDFNMPC_LIB=$R/_build/$v/libsdfnmpc.so timeout -k 10 120 python3 tools/vae_bench.py > $O/$v.txt 2>&1; done
grep -H "stem\|ms/encode  " $O/*.txt
