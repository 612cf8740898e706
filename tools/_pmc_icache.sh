#!/bin/bash
# Instruction-cache counters of the preparation kernels (sdf_mlp's 23.8k-instruction body against the
# shared SQC instruction cache), at 1 and 2.5 workgroup rounds (TILE 32, B from $BS); diagnostic.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out/pmcic; mkdir -p $O
for B in ${BS:-200 1024}; do
  TILE=32 B=$B timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH --kernel-trace --output-format csv -d $O/b$B -o p -- python3 $R/tools/sdf_prep_drv.py > /dev/null 2>> $O/err.log || { echo "pass $B failed"; tail -5 $O/err.log; exit 3; }
done
python3 - <<'PY'
import csv, glob, collections, os
O = os.environ.get("GRAFT_REPO_ROOT", "/root/repo") + "/gpurun_out/pmcic"
for d in sorted(glob.glob(O + "/b*")):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0].split("::")[-1]
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in acc.items():
        print(os.path.basename(d), k, {c: sum(v) / len(v) for c, v in cs.items()})
PY
