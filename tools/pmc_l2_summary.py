"""profiles/<round>/pmc_l2_prep.json from tools/_pmc_l2.sh output (gpurun_out/pmcl2): per kernel and SDF
tile size, the mean per dispatch of each counter, plus the derived L2-side traffic of sdf_mlp."""
import collections
import csv
import glob
import json
import os
import sys

base, out = sys.argv[1], sys.argv[2]
res = collections.defaultdict(dict)
for d in sorted(glob.glob(os.path.join(base, "p*_t*"))):
    tile = d.split("_t")[-1]
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(os.path.join(d, "p_counter_collection.csv"))):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0].split("::")[-1]
        acc[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
    for (k, c), v in acc.items():
        res[f"{k}@tile{tile}"][c] = sum(v) / len(v)
    dur = collections.defaultdict(list)
    for r in csv.DictReader(open(os.path.join(d, "p_kernel_trace.csv"))):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0].split("::")[-1]
        dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for k, v in dur.items():
        res[f"{k}@tile{tile}"].setdefault("duration_us_median", sorted(v)[len(v) // 2])
for key, c in res.items():
    if "TCP_TCC_READ_REQ_sum" in c:
        c["l2_to_cu_read_bytes_if_128B_req"] = 128.0 * c["TCP_TCC_READ_REQ_sum"]
    if "TCC_HIT_sum" in c and "TCC_MISS_sum" in c:
        c["tcc_hit_rate"] = c["TCC_HIT_sum"] / max(1.0, c["TCC_HIT_sum"] + c["TCC_MISS_sum"])
json.dump({"workload": "preparation phase, B=1024 x N=40 (tools/sdf_prep_drv.py), 5 launches per pass",
           "passes": ["TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum", "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum",
                      "FETCH_SIZE", "SQ_INSTS_VMEM_RD SQ_INSTS_MFMA SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES"],
           "kernels": res}, open(out, "w"), indent=1)
print(json.dumps({k: {c: round(v, 4) if isinstance(v, float) else v for c, v in d.items()} for k, d in res.items() if "sdf_mlp" in k}, indent=1))
