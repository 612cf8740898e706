#!/bin/bash
# Round profile on the GPU box: smoke, bench, rocprofv3 kernel-trace stats of the bench command,
# and separate FETCH_SIZE / WRITE_SIZE passes (MI355X_MICROARCH.md: they cannot share a pass).
set -euo pipefail
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/prof
mkdir -p $O
timeout -k 10 300 python -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 400 python $R/bench.py > $O/bench.json 2> $O/bench.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o bench -- \
    python $R/bench.py --no-cpu-baseline > $O/bench_traced.json 2> $O/trace.err
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/fetch -o p -- \
    python $R/bench.py --no-cpu-baseline --steps 10 --warmup 2 --rti-steps 2 > /dev/null 2> $O/fetch.err
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/write -o p -- \
    python $R/bench.py --no-cpu-baseline --steps 10 --warmup 2 --rti-steps 2 > /dev/null 2> $O/write.err
echo done
