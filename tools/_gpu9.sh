#!/bin/bash
set -euo pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_sdf_wide.py tests/test_gpu_sdf.py -x -q > gpurun_out/wide_tests.log 2>&1 || { tail -40 gpurun_out/wide_tests.log; exit 2; }
tail -3 gpurun_out/wide_tests.log
timeout -k 10 300 python tools/wide_bench.py 512 60 2>&1 | tee gpurun_out/wide_bench.log
