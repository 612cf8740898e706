#!/bin/bash
# LDS-side SQ counters of rti_qp_kernel (plain build, no stamps): bank conflicts, LDS instruction mix
set -euo pipefail
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out/pmcqp; mkdir -p $O
timeout -k 10 200 python3 $R/tools/qp_stamps.py > $O/stamps.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_LDS_ADDR_CONFLICT SQ_INSTS_VALU \
    --kernel-trace --output-format csv -d $O/p1 -o p -- $R/tools/_qp_plain_drv /tmp/qp_in.bin > $O/drv.log 2>&1
python3 - <<'PY'
import csv, glob, collections, os
O = os.environ.get("GRAFT_REPO_ROOT", "/root/repo") + "/gpurun_out/pmcqp"
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(O + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0].split("::")[-1]
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    print(k, {c: round(sum(v) / len(v)) for c, v in sorted(d.items())})
PY
