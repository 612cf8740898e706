#!/bin/bash
# Round profile on the GPU box: GPU tests, smoke, bench, rocprofv3 kernel-trace stats of the bench
# command, and separate FETCH_SIZE / WRITE_SIZE passes (MI355X_MICROARCH.md: they cannot share a pass).
set -euo pipefail
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/prof
mkdir -p $O
cd $R
timeout -k 10 600 python -m pytest tests -q -m gpu -x > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 2; }
tail -2 $O/pytest_gpu.log
cd /tmp
timeout -k 10 300 python -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 400 python $R/bench.py > $O/bench.json 2> $O/bench.err
cat $O/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o bench -- \
    python $R/bench.py --no-cpu-baseline --no-b1 > $O/bench_traced.json 2> $O/trace.err
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/fetch -o p -- \
    python $R/bench.py --no-cpu-baseline --steps 5 --warmup 2 --prep-steps 2 --no-b1 > /dev/null 2> $O/fetch.err
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/write -o p -- \
    python $R/bench.py --no-cpu-baseline --steps 5 --warmup 2 --prep-steps 2 --no-b1 > /dev/null 2> $O/write.err
echo done
