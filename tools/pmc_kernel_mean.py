#!/usr/bin/env python3
"""Mean per dispatch of every counter of one kernel over rocprofv3 --pmc output directories
(<dir>/**/p_counter_collection.csv), with the median kernel-trace duration:
    python3 tools/pmc_kernel_mean.py <kernel-name-substring> <dir> [<dir> ...]"""
import collections
import csv
import glob
import json
import os
import sys


def main():
    name, dirs = sys.argv[1], sys.argv[2:]
    acc, dur = collections.defaultdict(list), []
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                if name in r["Kernel_Name"]:
                    acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
        for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                if name in r["Kernel_Name"]:
                    dur.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    out = {c: sum(v) / len(v) for c, v in sorted(acc.items())}
    out["dispatches"] = max((len(v) for v in acc.values()), default=0)
    if dur:
        out["duration_us_median"] = sorted(dur)[len(dur) // 2]
    print(json.dumps({name: out}, indent=1))


if __name__ == "__main__":
    main()
