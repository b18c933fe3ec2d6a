#!/usr/bin/env python3
"""Summarise tools/gpu_bench_pmc.sh into profiles/<tag>_bench_pmc.json: per kernel of the
bench workload, the average duration (rocprofv3 --kernel-trace --stats) and every PMC
counter per dispatch (mean over the dispatches of each pass), plus the sha256 of the
librtmi.so that was profiled and of its render-kernel object build/rt_kernels.o (bench.py
accepts the profile when either equals the build it loads: a change elsewhere in the
library leaves the render kernel's code, and so its counters, unchanged).

    python tools/bench_pmc_summary.py gpurun_out/pmc_<tag> <tag>

HBM bytes (MI355X_MICROARCH.md, HBM/rocprofv3): FETCH_SIZE and WRITE_SIZE are KiB per
dispatch; FETCH_SIZE counts half the bytes of wide streaming reads on gfx950, so
fetch bytes = 2 x FETCH_SIZE x 1024; write bytes = WRITE_SIZE x 1024.
"""
import csv
import glob
import hashlib
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "reinforcement-light-rays-pathtracer_amd", "build", "librtmi.so")
RENDER_OBJ = os.path.join(ROOT, "reinforcement-light-rays-pathtracer_amd", "build", "rt_kernels.o")
KEYS = ("k_render", "k_cull")


def main():
    d, tag = sys.argv[1], sys.argv[2]
    out = {"tag": tag, "workload": "bench.py --steps 10 --warmup 2 (Cornell 512x512, 256 spp, spp_split 64)",
           "lib_sha256": hashlib.sha256(open(LIB, "rb").read()).hexdigest(),
           "render_obj_sha256": (hashlib.sha256(open(RENDER_OBJ, "rb").read()).hexdigest()
                                 if os.path.exists(RENDER_OBJ) else open(RENDER_OBJ + ".sha256").read().strip()),
           "kernels": {}}
    stats = glob.glob(os.path.join(d, "kt", "*kernel_stats.csv"))
    if stats:
        shutil.copy(stats[0], os.path.join(ROOT, "profiles", f"{tag}_bench_kernel_stats.csv"))
        for row in csv.DictReader(open(stats[0])):
            if any(k in row["Name"] for k in KEYS):
                out["kernels"].setdefault(row["Name"], {})["avg_ns"] = float(row["AverageNs"])
                out["kernels"][row["Name"]]["calls"] = int(row["Calls"])
    for f in sorted(glob.glob(os.path.join(d, "*", "*counter_collection.csv"))):
        acc = {}
        for row in csv.DictReader(open(f)):
            if not any(k in row["Kernel_Name"] for k in KEYS):
                continue
            acc.setdefault((row["Kernel_Name"], row["Counter_Name"]), []).append(float(row["Counter_Value"]))
        for (k, c), v in acc.items():
            e = out["kernels"].setdefault(k, {}).setdefault("per_dispatch", {})
            e[c] = sum(v) / len(v)
    for k, e in out["kernels"].items():
        c = e.get("per_dispatch", {})
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            e["hbm_bytes_per_dispatch"] = 2.0 * c["FETCH_SIZE"] * 1024.0 + c["WRITE_SIZE"] * 1024.0
        if "GRBM_GUI_ACTIVE" in c and "avg_ns" in e:
            e["clock_ghz"] = c["GRBM_GUI_ACTIVE"] / 8.0 / e["avg_ns"]
        if "SQ_INSTS_VALU" in c and "GRBM_GUI_ACTIVE" in c:
            e["valu_issue_frac"] = c["SQ_INSTS_VALU"] / (1024.0 * c["GRBM_GUI_ACTIVE"] / 8.0 / 2.0)
    path = os.path.join(ROOT, "profiles", f"{tag}_bench_pmc.json")
    with open(path, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
