#!/bin/bash
set -euo pipefail
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p $R/gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/vtrace -o v -- python $R/tools/vae_bench.py 512 > $R/gpurun_out/vtrace.log 2>&1
echo ok
