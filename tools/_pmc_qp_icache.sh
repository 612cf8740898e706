#!/bin/bash
# Instruction-cache and issue counters of the serial QP kernel (102 KB of code against the SQC instruction
# cache shared by two CUs) at B = 256 (one wave per CU) and B = 1024 (one per SIMD), N = $N; diagnostic.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out/pmcqpic; mkdir -p $O
for B in ${BS:-256 1024}; do
  B=$B N=${N:-40} DRV=_vf timeout -k 10 120 python3 $R/tools/qp_stamps.py > $O/time_b$B.txt 2>&1
  cp /tmp/qp_in.bin /tmp/qp_in_b$B.bin
  n=0
  for set in "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH" \
             "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM" \
             "SQ_IFETCH_LEVEL SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_LEVEL_VMEM SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INSTS_MFMA" \
             "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INST_LEVEL_LDS SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES TA_TA_BUSY TA_FLAT_READ_WAVEFRONTS"; do
    n=$((n+1))
    timeout -s KILL 90 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $O/b$B/p$n -o p -- $R/tools/_qp_stamps_drv_vf /tmp/qp_in_b$B.bin >> $O/log.txt 2>> $O/err.log || { echo "pass $B/$n failed"; tail -5 $O/err.log; exit 3; }
  done
done
python3 - <<'PY'
import csv, glob, collections, os
O = os.environ.get("GRAFT_REPO_ROOT", "/root/repo") + "/gpurun_out/pmcqpic"
for d in sorted(glob.glob(O + "/b*/")):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0].split("::")[-1]
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in acc.items():
        if k != "rti_qp_kernel": continue
        print(os.path.basename(d.rstrip("/")), k, {c: round(sum(v) / len(v)) for c, v in sorted(cs.items())})
PY
cat $O/time_b*.txt | grep kernel
