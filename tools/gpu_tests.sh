#!/bin/bash
# GPU test pass on the box: the -m gpu suite (verbose log), optional test selection in $1.
set -euo pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest ${1:-tests} -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 || { tail -60 gpurun_out/gpu_tests.log; exit 2; }
tail -3 gpurun_out/gpu_tests.log
grep -E "PASSED|FAILED" gpurun_out/gpu_tests.log | wc -l
