"""profiles/pmc_summary.json from rocprofv3 FETCH_SIZE / WRITE_SIZE passes (csv output).

FETCH_SIZE / WRITE_SIZE are kilobytes per dispatch (rocprofv3 derived metrics, TCC_EA0 requests).
gfx950 correction (MI355X_MICROARCH.md, HBM): FETCH_SIZE counts half of the bytes of 16-B-per-lane
streaming reads -> doubled; WRITE_SIZE is exact for 16-B stores, uncalibrated for narrower ones.
Usage: python tools/pmc_summary.py <fetch_counter_collection.csv> <write_counter_collection.csv> B N tile_rows [csv_out_dir]
"""
import collections
import csv
import json
import os
import sys


def kernel_sources_sha16(root):
    """sha256 (16 hex digits) over the HIP sources and headers of the product library, in name order."""
    import glob
    import hashlib
    h = hashlib.sha256()
    for f in sorted(glob.glob(os.path.join(root, "sdf-nmpc_amd", "csrc", "*.hip")) +
                    glob.glob(os.path.join(root, "sdf-nmpc_amd", "csrc", "*.h"))):
        with open(f, "rb") as fh:
            h.update(os.path.basename(f).encode() + b"\0" + fh.read())
    return h.hexdigest()[:16]


def _git_head(root):
    import subprocess
    try:
        return subprocess.run(["git", "-C", root, "rev-parse", "--short", "HEAD"], capture_output=True, text=True,
                              timeout=10).stdout.strip() or None
    except (OSError, subprocess.SubprocessError):
        return None


def per_kernel(path, counter):
    acc = collections.defaultdict(list)
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] == counter:
                name = row["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0]
                acc[name].append(float(row["Counter_Value"]) * 1024.0)
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main():
    fetch, write, B, N, tile = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
    fb, wb = per_kernel(fetch, "FETCH_SIZE"), per_kernel(write, "WRITE_SIZE")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = {"B": B, "N": N, "tile_rows": tile, "source": "rocprofv3 --pmc FETCH_SIZE | WRITE_SIZE (separate passes)",
           "correction": "fetch bytes = 2 x FETCH_SIZE (gfx950 16-B streaming reads); write bytes = WRITE_SIZE",
           # what the passes measured: the tree's commit when the summary was made, and a hash of the kernel
           # sources (bench.py compares it with the sources it runs, so a stale traffic figure is labelled)
           "commit": _git_head(root), "kernel_sources_sha16": kernel_sources_sha16(root),
           "kernels": {}}
    for k in sorted(set(fb) | set(wb)):
        f2 = 2.0 * fb.get(k, 0.0)
        out["kernels"][k.split("::")[-1].replace("_kernel", "")] = {
            "fetch_bytes_per_launch": f2, "write_bytes_per_launch": wb.get(k, 0.0),
            "hbm_bytes_per_launch": f2 + wb.get(k, 0.0)}
    with open(os.path.join(root, "profiles", "pmc_summary.json"), "w") as f:
        json.dump(out, f, indent=1)
    if len(sys.argv) > 6:  # per-kernel csv summaries (mean KB per dispatch) into this directory
        for path, counter, tag in ((fetch, "FETCH_SIZE", "fetch"), (write, "WRITE_SIZE", "write")):
            acc = collections.defaultdict(list)
            with open(path) as f:
                for row in csv.DictReader(f):
                    if row["Counter_Name"] == counter:
                        acc[row["Kernel_Name"].split("(")[0].replace("void ", "")].append(float(row["Counter_Value"]))
            with open(os.path.join(sys.argv[6], f"pmc_{tag}_per_kernel.csv"), "w") as f:
                f.write("kernel,counter,dispatches,mean_KB_per_dispatch\n")
                for k, v in sorted(acc.items()):
                    f.write(f'"{k}",{counter},{len(v)},{sum(v) / len(v):.3f}\n')
    for k, v in out["kernels"].items():
        print(f"{k:28s} fetch {v['fetch_bytes_per_launch'] / 1e6:10.3f} MB  write {v['write_bytes_per_launch'] / 1e6:10.3f} MB")


if __name__ == "__main__":
    main()
