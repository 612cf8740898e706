cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests -q -m gpu -x -k "qp or controller" > gpurun_out/pytest_qp.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_qp.log; [ $rc -gt 1 ] && exit $rc
timeout -k 10 200 python tools/qp_stamps.py > gpurun_out/stamps.log 2>&1 || { tail gpurun_out/stamps.log; exit 4; }
for v in ${VARIANTS:-b}; do timeout -k 10 100 tools/_qp_stamps_drv_$v /tmp/qp_in.bin 2>&1 | grep kernel | sed "s/^/$v: /" || exit 5; done
head -9 gpurun_out/stamps.log
