#!/bin/bash
# Quick GPU check: the -m gpu suite, then a short default bench run (no CPU baseline).
set -euo pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest ${1:-tests} -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/quick_tests.log 2>&1 || { tail -40 gpurun_out/quick_tests.log; exit 2; }
tail -2 gpurun_out/quick_tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/quick_bench.json 2> gpurun_out/quick_bench.err
python -c "import json; d=json.load(open('gpurun_out/quick_bench.json')); print(d['value'], d['ms_per_step'], d['p50_step_ms_b1'], d['qp_iters_max'], d['kernel_ms']); print('c2', d['c2']); print('c1', d.get('c1'))"
