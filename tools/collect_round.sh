#!/bin/bash
# Copy the round check's summaries (gpurun_out/rc/, tools/round_check.sh) into profiles/<round>/ and
# rebuild profiles/pmc_summary.json from its FETCH_SIZE / WRITE_SIZE passes.  CPU only.
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd); RC=$R/gpurun_out/rc; P=$R/profiles/${1:?round, e.g. r04}
mkdir -p $P
cp $RC/bench.json $P/bench_$1.json
cp $RC/bench_c5.json $P/bench_c5_$1.json
cp $RC/trace/bench_kernel_stats.csv $P/kernel_stats_bench.csv
cp $RC/trace_c5/bench_kernel_stats.csv $P/kernel_stats_c5.csv
[ -f $RC/pytest_gpu.log ] && cp $RC/pytest_gpu.log $P/pytest_gpu.log
[ -f $RC/smoke.log ] && cp $RC/smoke.log $P/smoke.log
python3 $R/tools/pmc_summary.py $RC/fetch/p_counter_collection.csv $RC/write/p_counter_collection.csv 1024 40 32 $P
ls $P
