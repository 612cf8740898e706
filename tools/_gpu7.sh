#!/bin/bash
# VAE encoder: GPU parity tests + timing
set -euo pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_vae.py -x -q > gpurun_out/vae_tests.log 2>&1 || { tail -40 gpurun_out/vae_tests.log; exit 2; }
tail -3 gpurun_out/vae_tests.log
timeout -k 10 300 python tools/vae_bench.py 512 2>&1 | tee gpurun_out/vae_bench.log
