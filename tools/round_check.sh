#!/bin/bash
# Round check on a fresh GPU box: the -m gpu suite, smoke, the default bench (C3 + c2 leg + CPU baseline),
# the C5 bench, rocprofv3 kernel-trace stats of both, FETCH_SIZE / WRITE_SIZE passes of the default bench
# (separate runs, MI355X_MICROARCH.md), and the QP per-phase cycle stamps.  Everything under
# gpurun_out/rc/; the summaries worth keeping are copied to profiles/<round>/ afterwards.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/rc
mkdir -p $O
cd $R
# PART=1: tests + smoke; PART=2: benches, traces, PMC passes; PART=3: QP stamps and sweeps (default: all)
PART=${PART:-all}
if [ "$PART" = all ] || [ "$PART" = 1 ]; then
timeout -k 10 900 python -u -m pytest tests -v -m gpu -x --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 2; }
tail -2 $O/pytest_gpu.log
cd /tmp
timeout -k 10 300 python -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
cat $O/smoke.log
fi
if [ "$PART" = all ] || [ "$PART" = 2 ]; then
cd /tmp
timeout -k 10 400 python $R/bench.py > $O/bench.json 2> $O/bench.err
cat $O/bench.json
timeout -k 10 400 python $R/bench.py --config c5 > $O/bench_c5.json 2> $O/bench_c5.err
cat $O/bench_c5.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o bench -- \
    python3 $R/bench.py --no-cpu-baseline --no-b1 --no-c2 --no-c1 --no-scene > $O/bench_traced.json 2> $O/trace.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c5 -o bench -- \
    python3 $R/bench.py --config c5 --no-cpu-baseline > $O/bench_c5_traced.json 2> $O/trace_c5.err
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/fetch -o p -- \
    python3 $R/bench.py --no-cpu-baseline --steps 5 --warmup 2 --prep-steps 2 --no-b1 --no-c2 --no-c1 --no-scene > /dev/null 2> $O/fetch.err
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/write -o p -- \
    python3 $R/bench.py --no-cpu-baseline --steps 5 --warmup 2 --prep-steps 2 --no-b1 --no-c2 --no-c1 --no-scene > /dev/null 2> $O/write.err
fi
if [ "$PART" = all ] || [ "$PART" = 3 ]; then
# the stamps driver is rebuilt from the current rti_qp.hip, so the stamps always describe this tree's kernel
(cd $R && timeout -k 10 300 hipcc --offload-arch=gfx950 -O3 -std=c++17 -w -mllvm -amdgpu-mfma-vgpr-form -mllvm -amdgpu-sched-strategy=max-ilp -DQP_STAMPS -I sdf-nmpc_amd/csrc \
    tools/qp_stamps_drv.hip sdf-nmpc_amd/csrc/rti_qp.hip -o tools/_qp_stamps_drv)
timeout -k 10 200 python3 $R/tools/qp_stamps.py > $O/qp_stamps.txt 2>&1
# the segmented kernel: per-phase stamps (P = 4, B = 64 and 1024) and the serial / segmented sweep over B and N
(cd $R && timeout -k 10 300 hipcc --offload-arch=gfx950 -O3 -std=c++17 -w -mllvm -amdgpu-mfma-vgpr-form -DSEG_STAMPS -I sdf-nmpc_amd/csrc \
    tools/seg_stamps_drv.hip sdf-nmpc_amd/csrc/rti_qp_seg.hip sdf-nmpc_amd/csrc/rti_qp.hip -o tools/_qp_stamps_drv_seg)
(cd $R && P=4 timeout -k 10 250 bash tools/seg_stamps.sh && cp gpurun_out/seg_stamps_b64.log $O/seg_stamps_b64.txt && cp gpurun_out/seg_stamps.log $O/seg_stamps_b1024.txt)
(cd $R && for n in 40 60; do N=$n timeout -k 10 120 python3 tools/seg_sweep_b.py 1 8 64 256 512 1024 || exit 1; done) > $O/qp_kernel_sweep.txt 2>&1
fi
echo done
