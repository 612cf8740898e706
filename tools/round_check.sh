#!/bin/bash
# Full round check on the GPU box: GPU tests, smoke, default bench, C5 bench, rocprofv3 kernel stats of both.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/rc
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -v -m gpu -x --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 2; }
tail -2 $O/pytest_gpu.log
cd /tmp
timeout -k 10 300 python -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
cat $O/smoke.log
timeout -k 10 400 python $R/bench.py > $O/bench.json 2> $O/bench.err
cat $O/bench.json
timeout -k 10 400 python $R/bench.py --config c5 > $O/bench_c5.json 2> $O/bench_c5.err
cat $O/bench_c5.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o bench -- \
    python $R/bench.py --no-cpu-baseline --no-b1 > $O/bench_traced.json 2> $O/trace.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c5 -o bench -- \
    python $R/bench.py --config c5 --no-cpu-baseline > $O/bench_c5_traced.json 2> $O/trace_c5.err
echo done
