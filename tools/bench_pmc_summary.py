#!/usr/bin/env python3
"""Summarise the rocprofv3 PMC passes of one bench workload (tools/gpu.sh pmc:<workload>)
into the profile bench.py reads for that workload's roofline.

    python tools/bench_pmc_summary.py gpurun_out/<tag>/pmc_<workload> <tag> <workload> [out_dir]

Output: profiles/<tag>_bench_pmc.json (cornell, the driver's workload) or
profiles/<tag>_<workload>_bench_pmc.json, holding
  * the profiled command (tools/gpu.sh bench_cmd: the bench's own command, so its frames are
    the bench's frames) with its --warmup / --steps,
  * the sha256 of librtmi.so and of the object file that holds the workload's kernels
    (bench.py accepts the profile when either equals the build it loads),
  * per kernel: every counter as the mean per dispatch and as the total per frame (frames
    split at the workload's marker kernel, in dispatch order), the PMC-pass durations
    (sq1's kernel trace: the counters slow the clock, so these are not the timing evidence --
    that is the counter-free kt summary, tools/gpu.sh kt:<workload>), and the clock the pass
    ran at (GRBM_GUI_ACTIVE / 8 / duration).

HBM bytes (MI355X_MICROARCH.md, HBM/rocprofv3): FETCH_SIZE and WRITE_SIZE are KiB per
dispatch, in separate passes, counted at the L2's fabric side (Infinity-Cache hits included).
FETCH_SIZE counts half the bytes of wide (16-B-per-lane) coalesced streaming reads on gfx950:
for kernels whose reads are such streams (the DQN forward's weight fragments, the frame
stores' read-for-ownership) fetch bytes = 2 x FETCH_SIZE x 1024 (fetch_scale 2).  Other access
widths are uncalibrated; the SARSA kernels read by gathers (grid lists, CDF rows, TD atomics)
and keep fetch_scale 1 -- their FETCH_SIZE is L2-miss traffic that the 256 MB Infinity Cache
largely serves (door_room's 170 MB map fits), not HBM bytes.  write bytes = WRITE_SIZE x 1024.
Profiles are keyed by the bench frame they ran (workload, width, height, spp, spp_split):
bench.py takes counters only from a profile of its own frame.
"""
import csv
import datetime
import glob
import hashlib
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(ROOT, "reinforcement-light-rays-pathtracer_amd", "build")
LIB = os.path.join(BUILD, "librtmi.so")

# profile name -> (kernel-name pattern kept, frame-marker pattern, object file of those kernels,
#                 bench arguments: must equal tools/gpu.sh bench_cmd, FETCH_SIZE scale)
# The BASELINE configs at their stated sizes: c1 (Cornell 256^2 x 4), cornell (= c2, the
# driver's line), door_room_sarsa (c3), archway_dqn (c4, 1024^2 x 512), complex_light (c5,
# 2048^2 x 1024 on one GPU); *_s16 / *_s64: the reduced-spp frames of earlier rounds.
WORKLOADS = {
    "cornell": (r"::k_render_ps<|::k_cull", r"::k_render_ps<", "rt_kernels.o",
                "--steps 4 --warmup 3 --cpu-seconds 0 --no-parity", 2),
    "cornell_c1": (r"::k_render_ps<|::k_cull", r"::k_render_ps<", "rt_kernels.o",
                   "--width 256 --height 256 --spp 4 --spp-split 4 --steps 20 --warmup 3 --cpu-seconds 0 "
                   "--no-parity", 2),
    # (the GPU preset's matrix-core renders run k_render_pq + k_fold_chunks; per-pixel k_render otherwise)
    "complex_light": (r"::k_render(_pq)?<|::k_fold_chunks", r"::k_render(_pq)?<", "rt_kernels.o",
                      "--workload complex_light --steps 1 --warmup 1 --cpu-seconds 0 --no-parity", 2),
    "complex_light_s64": (r"::k_render(_pq)?<|::k_fold_chunks", r"::k_render(_pq)?<", "rt_kernels.o",
                          "--workload complex_light --spp 64 --steps 2 --warmup 1 --cpu-seconds 0 --no-parity", 2),
    "door_room_sarsa": (r"::k_sarsa_", r"::k_sarsa_render(_pq)?<", "rt_sarsa.o",
                        "--workload door_room_sarsa --steps 4 --warmup 1 --cpu-seconds 0", 1),
    "archway_dqn": (r"::k_dqn_", r"::k_dqn_frame_begin", "rt_dqn.o",
                    "--workload archway_dqn --steps 1 --warmup 1 --cpu-seconds 0", 2),
    "archway_dqn_s16": (r"::k_dqn_", r"::k_dqn_frame_begin", "rt_dqn.o",
                        "--workload archway_dqn --spp 16 --steps 2 --warmup 1 --cpu-seconds 0", 2),
}

# bench.py's per-workload frame defaults (width, height, spp, spp_split)
BENCH_FRAMES = {"cornell": (512, 512, 256, 64), "door_room_sarsa": (512, 512, 256, 64),
                "archway_dqn": (1024, 1024, 512, 1), "complex_light": (2048, 2048, 1024, 32)}


def frame_of_args(args: str):
    """(workload, width, height, spp, spp_split) of a bench argument string"""
    def opt(name, default):
        m = re.search(rf"--{name} (\S+)", args)
        return m.group(1) if m else default
    wl = opt("workload", "cornell")
    W, H, spp, split = BENCH_FRAMES[wl]
    return (wl, int(opt("width", W)), int(opt("height", H)), int(opt("spp", spp)), int(opt("spp-split", split)))


def sha(path):
    if os.path.exists(path):
        return hashlib.sha256(open(path, "rb").read()).hexdigest()
    return open(path + ".sha256").read().strip() if os.path.exists(path + ".sha256") else ""


def family(name):
    """'void rt::(anonymous namespace)::k_dqn_bounce<0>(rt::DqnLaunch, int)' -> 'k_dqn_bounce<0>'"""
    m = re.search(r"::(k_[a-z0-9_]+(<[^>]*>)?)\(", name)
    return m.group(1) if m else name


def frames_of(rows, keep, marker):
    """rows of one pass in dispatch order -> list of frames, each a list of kept rows"""
    frames = []
    for r in rows:
        if re.search(marker, r["Kernel_Name"]):
            frames.append([])
        if frames and re.search(keep, r["Kernel_Name"]):
            frames[-1].append(r)
    return frames


def main():
    if sys.argv[1] == "--args":  # the profiled bench arguments of a workload (tools/gpu.sh)
        print(WORKLOADS[sys.argv[2]][3])
        return
    d, tag = sys.argv[1], sys.argv[2]
    wl = sys.argv[3] if len(sys.argv) > 3 else "cornell"
    keep, marker, obj, args, fetch_scale = WORKLOADS[wl]
    w = re.search(r"--warmup (\d+)", args)
    s = re.search(r"--steps (\d+)", args)
    bench_wl, fw, fh, fspp, fsplit = frame_of_args(args)
    out = {"tag": tag, "workload_name": bench_wl, "profile_name": wl, "command": "python3 bench.py " + args,
           "frame": {"width": fw, "height": fh, "spp": fspp, "spp_split": fsplit}, "fetch_scale": fetch_scale,
           "warmup": int(w.group(1)), "steps": int(s.group(1)),
           "created": datetime.datetime.now(datetime.timezone.utc).isoformat(timespec="seconds"),
           "lib_sha256": sha(LIB), "obj": obj, "obj_sha256": sha(os.path.join(BUILD, obj)), "kernels": {}}
    if wl == "cornell":  # the key earlier bench.py versions matched on
        out["render_obj_sha256"] = out["obj_sha256"]
    n_frames = None
    owner = {}  # counter -> the pass it is taken from (GRBM_GUI_ACTIVE is in two passes)
    for f in sorted(glob.glob(os.path.join(d, "*", "*counter_collection.csv"))):
        rows = list(csv.DictReader(open(f)))
        # one row per (dispatch, counter): group into dispatches
        disp = {}
        for r in rows:
            e = disp.setdefault(int(r["Dispatch_Id"]), {"Kernel_Name": r["Kernel_Name"], "c": {}})
            e["c"][r["Counter_Name"]] = e["c"].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        ordered = [disp[k] for k in sorted(disp)]
        frames = frames_of(ordered, keep, marker)
        n_frames = len(frames) if n_frames is None else min(n_frames, len(frames))
        for fi, fr in enumerate(frames):
            for r in fr:
                k = out["kernels"].setdefault(family(r["Kernel_Name"]), {"per_dispatch": {}, "per_frame": [], "_n": {}})
                while len(k["per_frame"]) <= fi:
                    k["per_frame"].append({})
                for c, v in r["c"].items():
                    if owner.setdefault(c, f) != f:
                        continue
                    k["per_frame"][fi][c] = k["per_frame"][fi].get(c, 0.0) + v
                    k["per_dispatch"][c] = k["per_dispatch"].get(c, 0.0) + v
                    k["_n"][c] = k["_n"].get(c, 0) + 1
    for k in out["kernels"].values():
        for c in k["per_dispatch"]:
            k["per_dispatch"][c] /= k["_n"][c]
        del k["_n"]
    # durations of the sq1 pass (the one with GRBM_GUI_ACTIVE), per frame
    for f in glob.glob(os.path.join(d, "sq1", "*kernel_trace.csv")):
        rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Dispatch_Id"]))
        for fi, fr in enumerate(frames_of(rows, keep, marker)):
            for r in fr:
                k = out["kernels"].get(family(r["Kernel_Name"]))
                if k is None or fi >= len(k["per_frame"]):
                    continue
                ns = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
                k["per_frame"][fi]["duration_ns"] = k["per_frame"][fi].get("duration_ns", 0.0) + ns
                k.setdefault("_dur", []).append(ns)
    for k in out["kernels"].values():
        dur = k.pop("_dur", [])
        if dur:
            k["avg_ns"] = sum(dur) / len(dur)
            k["calls"] = len(dur)
        c = k["per_dispatch"]
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            k["hbm_bytes_per_dispatch"] = fetch_scale * c["FETCH_SIZE"] * 1024.0 + c["WRITE_SIZE"] * 1024.0
        for fr in k["per_frame"]:
            if "FETCH_SIZE" in fr and "WRITE_SIZE" in fr:
                fr["hbm_bytes"] = fetch_scale * fr["FETCH_SIZE"] * 1024.0 + fr["WRITE_SIZE"] * 1024.0
            if "GRBM_GUI_ACTIVE" in fr and fr.get("duration_ns"):
                fr["clock_ghz"] = fr["GRBM_GUI_ACTIVE"] / 8.0 / fr["duration_ns"]
        if "GRBM_GUI_ACTIVE" in c and "avg_ns" in k:
            k["clock_ghz"] = c["GRBM_GUI_ACTIVE"] / 8.0 / k["avg_ns"]
        if "SQ_INSTS_VALU" in c and "GRBM_GUI_ACTIVE" in c:
            k["valu_issue_frac"] = c["SQ_INSTS_VALU"] / (1024.0 * c["GRBM_GUI_ACTIVE"] / 8.0 / 2.0)
    out["frames"] = n_frames or 0
    # (on the GPU box: into gpurun_out/<tag>/profiles/, which gpurun copies back; tools/gpu.sh
    # collect:<tag> moves it to profiles/ here)
    odir = sys.argv[4] if len(sys.argv) > 4 else os.path.join(ROOT, "profiles")
    os.makedirs(odir, exist_ok=True)
    path = os.path.join(odir, f"{tag}_bench_pmc.json" if wl == "cornell" else f"{tag}_{wl}_bench_pmc.json")
    with open(path, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps({k: (v if k != "kernels" else sorted(v)) for k, v in out.items()}))


if __name__ == "__main__":
    main()
