cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -q -m gpu -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail gpurun_out/bench.err; exit 3; }
cat gpurun_out/bench.json
timeout -k 10 200 python tools/qp_stamps.py > gpurun_out/stamps.log 2>&1 || { tail gpurun_out/stamps.log; exit 4; }
cat gpurun_out/stamps.log
