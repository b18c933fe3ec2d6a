#!/usr/bin/env python3
"""Summarise tools/gpu_bench_pmc.sh into profiles/<tag>_bench_pmc.json: per kernel of the
bench workload, the average duration (rocprofv3 --kernel-trace --stats) and every PMC
counter per dispatch (mean over the dispatches of each pass), plus the sha256 of the
librtmi.so that was profiled and of its render-kernel object build/rt_kernels.o (bench.py
accepts the profile when either equals the build it loads: a change elsewhere in the
library leaves the render kernel's code, and so its counters, unchanged).

    python tools/bench_pmc_summary.py gpurun_out/<tag>/pmc_<workload> <tag> [<workload>]

The default workload (cornell) writes profiles/<tag>_bench_pmc.json, the others
profiles/<tag>_<workload>_bench_pmc.json; bench.py picks the profile whose "workload_name"
and object hash match the run.

HBM bytes (MI355X_MICROARCH.md, HBM/rocprofv3): FETCH_SIZE and WRITE_SIZE are KiB per
dispatch; FETCH_SIZE counts half the bytes of wide streaming reads on gfx950, so
fetch bytes = 2 x FETCH_SIZE x 1024; write bytes = WRITE_SIZE x 1024.
"""
import csv
import glob
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "reinforcement-light-rays-pathtracer_amd", "build", "librtmi.so")
BUILD = os.path.join(ROOT, "reinforcement-light-rays-pathtracer_amd", "build")
# workload -> (kernel-name substrings kept, the object file that holds those kernels, bench command)
WORKLOADS = {
    "cornell": (("k_render", "k_cull"), "rt_kernels.o",
                "bench.py --steps 4 --warmup 3 --cpu-seconds 0 --no-parity (Cornell 512x512, 256 spp, spp_split 64)"),
    "complex_light": (("k_render",), "rt_kernels.o",
                      "bench.py --workload complex_light --spp 64 --steps 4 --warmup 1 (2048x2048, 64 spp)"),
    "door_room_sarsa": (("k_sarsa",), "rt_sarsa.o",
                        "bench.py --workload door_room_sarsa --steps 4 --warmup 1 (512x512, 256 spp; frames 1-5)"),
    "archway_dqn": (("k_dqn",), "rt_dqn.o",
                    "bench.py --workload archway_dqn --spp 16 --steps 4 --warmup 1 (1024x1024, 16 spp)"),
}


def obj_sha(name):
    path = os.path.join(BUILD, name)
    if os.path.exists(path):
        return hashlib.sha256(open(path, "rb").read()).hexdigest()
    return open(path + ".sha256").read().strip() if os.path.exists(path + ".sha256") else ""


def main():
    d, tag = sys.argv[1], sys.argv[2]
    wl = sys.argv[3] if len(sys.argv) > 3 else "cornell"
    keys, obj, cmd = WORKLOADS[wl]
    out = {"tag": tag, "workload_name": wl, "workload": cmd,
           "lib_sha256": hashlib.sha256(open(LIB, "rb").read()).hexdigest(),
           "obj": obj, "obj_sha256": obj_sha(obj),
           "kernels": {}}
    if wl == "cornell":  # the name earlier bench.py versions match on
        out["render_obj_sha256"] = out["obj_sha256"]
    # PMC-pass kernel durations (the counters slow the clock: not the timing evidence --
    # that is the counter-free kt_<workload> summary, tools/gpu.sh kt:<workload>)
    for f in sorted(glob.glob(os.path.join(d, "*", "*counter_collection.csv"))):
        acc, disp = {}, {}
        for row in csv.DictReader(open(f)):
            if not any(k in row["Kernel_Name"] for k in keys):
                continue
            acc.setdefault((row["Kernel_Name"], row["Counter_Name"]), []).append(float(row["Counter_Value"]))
        for (k, c), v in acc.items():
            e = out["kernels"].setdefault(k, {}).setdefault("per_dispatch", {})
            e[c] = sum(v) / len(v)
    for f in sorted(glob.glob(os.path.join(d, "*", "*kernel_trace.csv"))):
        if not f.endswith("sq1_kernel_trace.csv"):
            continue
        dur = {}
        for row in csv.DictReader(open(f)):
            if any(k in row["Kernel_Name"] for k in keys):
                dur.setdefault(row["Kernel_Name"], []).append(
                    float(row["End_Timestamp"]) - float(row["Start_Timestamp"]))
        for k, v in dur.items():
            out["kernels"].setdefault(k, {}).update({"avg_ns": sum(v) / len(v), "calls": len(v)})
    for k, e in out["kernels"].items():
        c = e.get("per_dispatch", {})
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            e["hbm_bytes_per_dispatch"] = 2.0 * c["FETCH_SIZE"] * 1024.0 + c["WRITE_SIZE"] * 1024.0
        if "GRBM_GUI_ACTIVE" in c and "avg_ns" in e:
            e["clock_ghz"] = c["GRBM_GUI_ACTIVE"] / 8.0 / e["avg_ns"]
        if "SQ_INSTS_VALU" in c and "GRBM_GUI_ACTIVE" in c:
            e["valu_issue_frac"] = c["SQ_INSTS_VALU"] / (1024.0 * c["GRBM_GUI_ACTIVE"] / 8.0 / 2.0)
    path = os.path.join(ROOT, "profiles", f"{tag}_bench_pmc.json" if wl == "cornell"
                        else f"{tag}_{wl}_bench_pmc.json")
    with open(path, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
