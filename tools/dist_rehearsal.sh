#!/bin/bash
# Multi-rank bench rehearsal on a 1-GPU box: 2 ranks over gloo sharing cuda:0 (the driver's N>1 runs use one
# rank per GPU over RCCL); checks the launch protocol, sharding, barrier / max-over-ranks timing and output.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out
export SDFNMPC_DIST_BACKEND=gloo
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 \
    bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu-baseline --no-b1 --no-c1 --no-c2 --prep-steps 5 > gpurun_out/dist2.json 2> gpurun_out/dist2.err
python -c "import json; d=json.load(open('gpurun_out/dist2.json')); print(d['n_gpus'], d['value'], d['ms_per_step'], d['config']['global_batch'], d['qp_converged_frac'])"
