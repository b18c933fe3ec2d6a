#!/usr/bin/env python3
"""Summarise a tools/gpu_profile.sh run into profiles/: per-kernel average duration
(rocprofv3 --kernel-trace --stats) and HBM traffic per launch from the separate
FETCH_SIZE / WRITE_SIZE passes.

    python tools/pmc_summary.py gpurun_out/prof_<tag> <tag> [kernel-substring]

FETCH_SIZE / WRITE_SIZE are reported by rocprofv3 in KiB per dispatch.  MI355X_MICROARCH.md
(HBM, gfx950): FETCH_SIZE counts half the bytes of wide coalesced reads -> fetch bytes =
2 x FETCH_SIZE; WRITE_SIZE is exact for 16-B-per-lane stores.  Writes
profiles/<tag>_kernel_stats.csv (copy) and profiles/<tag>_pmc.json.
"""
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_kernel(path, counter):
    vals = {}
    for row in csv.DictReader(open(path)):
        if row["Counter_Name"] != counter:
            continue
        vals.setdefault(row["Kernel_Name"], []).append(float(row["Counter_Value"]))
    return vals


def main():
    d, tag = sys.argv[1], sys.argv[2]
    key = sys.argv[3] if len(sys.argv) > 3 else "k_render"
    out = {"tag": tag, "kernel_filter": key, "kernels": {}}
    stats = glob.glob(os.path.join(d, "kt", "*kernel_stats.csv"))
    if stats:
        shutil.copy(stats[0], os.path.join(ROOT, "profiles", f"{tag}_kernel_stats.csv"))
        for row in csv.DictReader(open(stats[0])):
            out["kernels"].setdefault(row["Name"], {})["avg_ns"] = float(row["AverageNs"])
            out["kernels"][row["Name"]]["calls"] = int(row["Calls"])
    for name, counter in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
        f = glob.glob(os.path.join(d, name, "*counter_collection.csv"))
        if not f:
            continue
        for k, v in per_kernel(f[0], counter).items():
            e = out["kernels"].setdefault(k, {})
            e[counter + "_kib_avg"] = sum(v) / len(v)
            e[counter + "_dispatches"] = len(v)
    for k, e in out["kernels"].items():
        if "FETCH_SIZE_kib_avg" in e and "WRITE_SIZE_kib_avg" in e:
            e["fetch_bytes"] = 2.0 * e["FETCH_SIZE_kib_avg"] * 1024.0
            e["write_bytes"] = e["WRITE_SIZE_kib_avg"] * 1024.0
            e["traffic_bytes_per_launch"] = e["fetch_bytes"] + e["write_bytes"]
    sel = {k: e for k, e in out["kernels"].items() if key in k}
    out["selected"] = sel
    with open(os.path.join(ROOT, "profiles", f"{tag}_pmc.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(sel, indent=1))


if __name__ == "__main__":
    main()
