#!/bin/bash
# SQ-side counters of the VAE stem kernel (where its waves spend their cycles): one rocprofv3 pass per set.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out/pmcstem; mkdir -p $O
n=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_VALU_MFMA_BUSY_CYCLES" \
           "SQ_WAVES SQ_INSTS_MFMA SQ_LDS_ADDR_CONFLICT SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_RD SQ_INST_LEVEL_VMEM SQ_LDS_IDX_ACTIVE" \
           "TA_TA_BUSY TA_FLAT_READ_WAVEFRONTS SQ_WAIT_INST_ANY SQ_INSTS_VMEM SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_FLAT"; do
  n=$((n+1))
  timeout -s KILL 60 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $O/p$n -o p -- python3 $R/tools/vae_bench.py 64 > /dev/null 2>> $O/err.log || { echo "pass $n failed"; tail -5 $O/err.log; exit 3; }
done
python3 - <<'PY'
import csv, glob, collections, os
O = os.environ.get("GRAFT_REPO_ROOT", "/root/repo") + "/gpurun_out/pmcstem"
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(O + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0].split("::")[-1]
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    if "vae_stem" not in k and "vae_conv" not in k: continue
    print(k, {c: round(sum(v) / len(v)) for c, v in sorted(d.items())})
PY
