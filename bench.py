#!/usr/bin/env python3
"""Benchmark: ray casts per second of the path tracer's hot path on BASELINE.json's configs.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload cornell|door_room_sarsa|
                    archway_dqn|complex_light] [--width .. --height .. --spp .. --spp-split ..]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

`python bench.py --gpus N` (N > 1, no WORLD_SIZE in the environment) starts the N ranks itself
under torch.distributed.run, one per GPU of the node, and relays rank 0's line; under a
launcher, WORLD_SIZE must equal --gpus.

Default workload (the driver's bench line): BASELINE config 2, the reference's Cornell box,
512x512, 256 spp, CPU-engine preset (cap 2 bounces, hit rule of the prebuilt CPU object,
uniform hemisphere sampling).  A step renders one full frame.  The other workloads are
BASELINE configs 3-5 for torchrun runs at more GPUs (a step = one frame; SARSA frames learn,
so their TD sums are all-reduced between ranks every step).

Multi-GPU: the frame is cut into 32x32 tiles dealt to the ranks by diagonals (rtmi.tiles; one
process per GPU); each rank renders its tiles with the HIP kernels, and the per-rank tile
buffers are gathered to rank 0 over RCCL into the full image -- asynchronously, into one of two
buffers, so frame i+1 renders while frame i is exchanged.  The frame is fixed as N grows:
strong scaling.

value = total ray casts (all ranks) / max-over-ranks wall time of the K timed steps, in
Mrays/s.  rank 0 prints one JSON line with the roofline of the render kernels (HIP events on
the launch stream; instruction and HBM counts from the committed rocprofv3 profile of the
same build, profiles/*_bench_pmc.json), the bit-exactness of 8 full 32x32 tiles (image and
ray casts) vs the CPU restatement, and the CPU baseline (oracle/, this host's cores, bounded
sample, best of 3).
"""
from __future__ import annotations

import argparse
import glob
import hashlib
import json
import os
import re
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))


def launch_command(argv, n: int):
    """The torch.distributed.run command that starts n ranks of this script (one per GPU of
    this node) with the same arguments.  --standalone: the launcher's own rendezvous store
    binds a free port and keeps it (no probe-then-close race for the port); --local-addr pins
    the address the ranks meet on to 127.0.0.1."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--standalone", "--local-addr=127.0.0.1", os.path.abspath(__file__)] + list(argv)


def rank_launch(argv, env) -> int | None:
    """`--gpus N`: with WORLD_SIZE unset and N > 1 this process becomes the launcher -- it
    starts N ranks under torch.distributed.run as a child process (nothing here has touched
    the GPU), waits, and returns their exit code (rank 0 prints the JSON line); None: run the
    bench in this process.  A WORLD_SIZE that differs from --gpus is refused (exit code 2)."""
    ap = argparse.ArgumentParser(add_help=False)
    ap.add_argument("--gpus", type=int, default=1)
    n = ap.parse_known_args(argv)[0].gpus
    if n < 1:
        print(f"bench.py: --gpus {n}: need at least one GPU", file=sys.stderr)
        return 2
    ws = env.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != n:
            print(f"bench.py: WORLD_SIZE={ws} but --gpus {n}: launch one rank per GPU "
                  f"(--nproc-per-node {n}) or drop the launcher", file=sys.stderr)
            return 2
        return None
    if n == 1:
        return None
    cmd = launch_command(argv, n)
    if env.get("RTMI_BENCH_DRY_RUN") == "1":  # (tests: the command, not the run)
        print(json.dumps(cmd))
        return 0
    return subprocess.run(cmd, env=dict(env)).returncode


if __name__ == "__main__":
    _rc = rank_launch(sys.argv[1:], os.environ)
    if _rc is not None:
        sys.exit(_rc)

import numpy as np  # noqa: E402

sys.path.insert(0, os.path.join(ROOT, "reinforcement-light-rays-pathtracer_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import rtmi  # noqa: E402

MODELS = os.path.join(ROOT, "assets", "models")
TILE = 32
# MI355X peaks (MI355X_MICROARCH.md): 1024 SIMD-32 units, one wave64 VALU instruction per
# 2 cycles each at the 2.4 GHz maximum clock; FP32 vector 157.3 TFLOP/s; HBM3E 8 TB/s.
VALU_ISSUE_PEAK_G = 1024 * 2.4 / 2.0  # G wave-instructions / s
VALU_PEAK_TFLOPS = 157.3
HBM_PEAK_GBS = 8000.0
MFMA_BF16_PEAK_TFLOPS = 2500.0  # dense bf16 (MI355X_MICROARCH.md; no sparsity)

WORKLOADS = {
    # name: (scene, preset, sampler, width, height, spp, spp_split, BASELINE config)
    "cornell": ("cornell", rtmi.RT_PRESET_CPU, "uniform", 512, 512, 256, 64, 2),
    # (config 3: spp_split 64 -- 4-sample work items balance the persistent queue's lanes: frames
    # 1-10 91.9 vs 102.6 ms at split 8 on one GPU, and each rank's launch at P = 8, where split 8
    # leaves about one item per lane: 6.5x vs 4.8x predicted, profiles/r5h/)
    "door_room_sarsa": ("door_room", rtmi.RT_PRESET_GPU, "sarsa", 512, 512, 256, 64, 3),
    "archway_dqn": ("archway", rtmi.RT_PRESET_GPU, "dqn", 1024, 1024, 512, 1, 4),
    # (config 5: spp_split 32 -- 2-sample chunks end each rank's launch of the P = 8 split
    # sooner: 121.6 vs 131.3 ms per rank set at 64 spp, profiles/r3ag/; one GPU unchanged)
    "complex_light": ("complex_light_room", rtmi.RT_PRESET_GPU, "uniform", 2048, 2048, 1024, 32, 5),
}
# the roofline's dominant kernel per workload: (rt_ktime family timed live, its name in the
# profiles, bound, object file holding it -- the profile must come from the same object)
ROOF = {
    "cornell": (rtmi.RT_KT_RENDER_PS, "k_render_ps<", "valu", "rt_kernels.o"),
    "complex_light": (rtmi.RT_KT_RENDER, "k_render<", "valu", "rt_kernels.o"),
    "door_room_sarsa": (rtmi.RT_KT_SARSA_RENDER, "k_sarsa_render<", "valu", "rt_sarsa.o"),
    "archway_dqn": (rtmi.RT_KT_DQN_MLP, "k_dqn_mlp<", "mfma", "rt_dqn.o"),
}
# the kernels a timed family launches (rt_ktime times the launcher, so its time covers them
# all): the persistent GPU-preset and SARSA renders and their folds (k_render_pq,
# k_fold_chunks; k_sarsa_render_pq, k_sarsa_fold) count with k_render / k_sarsa_render
FAMILY_RE = {
    "k_render<": r"^k_render(_pq)?<|^k_fold_chunks$",
    "k_sarsa_render<": r"^k_sarsa_render(_pq)?<|^k_sarsa_fold$",
}


def family_re(kernel: str) -> str:
    """profile-key pattern of the kernels behind a family name ('k_x<' or 'k_x')"""
    if kernel in FAMILY_RE:
        return FAMILY_RE[kernel]
    base = re.escape(kernel.rstrip("<"))
    return rf"^{base}(<|$)"
# committed rocprofv3 PMC profiles (tools/gpu.sh pmc:<workload> -> tools/bench_pmc_summary.py)
PMC_GLOB = os.path.join(ROOT, "profiles", "*_bench_pmc.json")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None, help="timed frames (default: 20 for cornell, else 10)")
    ap.add_argument("--warmup", type=int, default=None,
                    help="untimed frames first (default: 10 for cornell -- the clock ramps over the first "
                         "~40 ms of a 4-ms frame stream -- else 1)")
    ap.add_argument("--workload", default="cornell", choices=sorted(WORKLOADS))
    ap.add_argument("--width", type=int, default=None)
    ap.add_argument("--height", type=int, default=None)
    ap.add_argument("--spp", type=int, default=None)
    ap.add_argument("--spp-split", type=int, default=None)
    ap.add_argument("--cpu-seconds", type=float, default=8.0,
                    help="target duration of one CPU-baseline run (best of 3; 0 disables)")
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--emulate-ranks", type=int, default=0,
                    help="P > 1: on one GPU, run each of the P ranks' tile sets through the timed loop in turn "
                         "(host work included; a device copy stands in for the gather) and predict the P-GPU step")
    args = ap.parse_args()
    if args.steps is None:
        args.steps = 20 if args.workload == "cornell" else 10
    if args.warmup is None:
        args.warmup = 10 if args.workload == "cornell" else 1
    return args


def lib_sha256() -> str:
    return hashlib.sha256(open(rtmi.LIB_PATH, "rb").read()).hexdigest()


def obj_sha256(name: str) -> str:
    """sha256 of build/<name>, or the hash the Makefile wrote beside it (object files do not
    travel to the GPU box)."""
    path = os.path.join(os.path.dirname(rtmi.LIB_PATH), name)
    if os.path.exists(path):
        return hashlib.sha256(open(path, "rb").read()).hexdigest()
    if os.path.exists(path + ".sha256"):
        return open(path + ".sha256").read().strip()
    return ""


def profile_frame(prof):
    """(width, height, spp, spp_split) of the frame a profile ran: its "frame" record, or
    (older profiles) its bench command over the workload's defaults"""
    f = prof.get("frame")
    if f:
        return (f["width"], f["height"], f["spp"], f["spp_split"])
    _, _, _, W, H, spp, split, _ = WORKLOADS[prof.get("workload_name", "cornell")]
    cmd = prof.get("command", "")

    def opt(name, default):
        m = re.search(rf"--{name} (\S+)", cmd)
        return int(m.group(1)) if m else default
    return (opt("width", W), opt("height", H), opt("spp", spp), opt("spp-split", split))


def load_profile(workload: str, frame):
    """The committed PMC profile of this workload, frame (width, height, spp, spp_split) and
    build: its library hash equals the loaded librtmi.so, or the hash of the object holding
    the workload's kernels equals the one this library was linked from (a change elsewhere
    leaves those kernels' code, and so their counters, unchanged).  Among several, the newest
    by the profile's own creation stamp (then its file name); without a match, the newest of
    the workload and frame, flagged; a profile of another frame is never used."""
    sha, osha = lib_sha256(), obj_sha256(ROOF[workload][3])
    best = None
    for path in glob.glob(PMC_GLOB):
        try:
            prof = json.load(open(path))
        except (OSError, ValueError):
            continue
        if prof.get("workload_name", "cornell") != workload or profile_frame(prof) != tuple(frame):
            continue
        psha = prof.get("obj_sha256") or prof.get("render_obj_sha256")
        match = prof.get("lib_sha256") == sha or bool(osha and psha == osha)
        key = (match, prof.get("created", ""), os.path.basename(path))
        if best is None or key > best[0]:
            best = (key, os.path.relpath(path, ROOT), prof)
    return (best[1], best[2], best[0][0]) if best else (None, None, False)


def frame_counters(prof, kernel: str, warmup: int, steps: int):
    """Counters of the kernel per frame: the profiled frames [warmup, warmup + steps) when the
    profile ran the bench's own frames (learning workloads differ frame to frame), else the
    mean over its frames; old profiles: the per-dispatch means (one launch per frame)."""
    ks = [k for k in prof["kernels"] if re.search(family_re(kernel), k.split("::")[-1])]
    per = {}
    matched = False
    for k in ks:
        e = prof["kernels"][k]
        fr = e.get("per_frame")
        if fr:
            if prof.get("warmup") == warmup and prof.get("steps") == steps and len(fr) >= warmup + steps:
                sel, matched = fr[warmup:warmup + steps], True
            else:
                sel = fr
            for f in sel:
                for c, v in f.items():
                    per[c] = per.get(c, 0.0) + v / len(sel)
        else:
            for c, v in e.get("per_dispatch", {}).items():
                per[c] = per.get(c, 0.0) + v
            if "hbm_bytes_per_dispatch" in e:
                per["hbm_bytes"] = per.get("hbm_bytes", 0.0) + e["hbm_bytes_per_dispatch"]
            if "avg_ns" in e:
                per["duration_ns"] = per.get("duration_ns", 0.0) + e["avg_ns"]
    return per, matched


def roofline(args, geom, params, casts_per_frame: float, kt: dict):
    """Roofline of the workload's dominant kernel.

    Time: that kernel's launches in the timed steps, HIP events on its own launch stream
    (rt_ktime_*), per frame.  Work: the committed rocprofv3 profile of the same build and
    workload (tools/gpu.sh pmc:<workload>), per frame.
    * VALU-bound kernels (k_render_ps, k_render, k_sarsa_render): frac = VALU
      wave-instructions / (time x 1024 SIMDs x one wave-instruction per 2 cycles at 2.4 GHz).
      Their triangle records are scalar-cache resident; HBM traffic is the frame (profile).
    * The DQN forward k_dqn_mlp (a dense contraction): frac = the bf16 MFMA flops the kernel
      executes (SQ_INSTS_VALU_MFMA_BF16 x 16384 per v_mfma_f32_16x16x32_bf16, from the profile)
      / time / the 2.5 PF dense bf16 peak, the matrix pipe's busy fraction beside it; the
      reference's algorithmic flops (2 sum(in x out) per ray per NN bounce, SURVEY.md §8(d), with
      the 918-wide layer 0 the kernel folds to a 3-wide affine map) as a named extra.
    Informational for the scan kernels: the reference's brute-force flops (71 per
    ray-triangle test) per second and the north star's HBM-algorithmic ratio (36 B per
    triangle per cast as if streamed: not a bound on these kernels)."""
    fam, kname, bound, _ = ROOF[args.workload]
    steps = args.steps
    if not kt[fam][1]:  # (this configuration ran another kernel family: the one that took the time)
        fam = max(kt, key=lambda f: kt[f][0])
        kname = rtmi.ktime_name(fam) + "<"
    t = kt[fam][0] / steps * 1e-3  # s per frame in the dominant kernel
    if t <= 0.0:
        return {"bound": bound, "achieved": None, "frac": None, "traffic": None, "kernel": None}
    path, prof, match = load_profile(args.workload, (params.width, params.height, params.spp, params.spp_split))
    line = {"bound": bound, "achieved": None, "frac": None, "traffic": None, "kernel": kname.rstrip("<"),
            "kernel_ms": round(t * 1e3, 4), "kernel_launches_per_step": kt[fam][1] / steps,
            "profile": path, "profile_matches_build": match}
    if bound == "valu":
        line.update({"peak": VALU_ISSUE_PEAK_G, "unit": "G VALU wave-instr/s"})
    else:
        line.update({"peak": MFMA_BF16_PEAK_TFLOPS, "unit": "TFLOP/s"})
    # every timed kernel family's share of the frame's kernel time
    tot = sum(v[0] for v in kt.values())
    line["kernel_share"] = round(kt[fam][0] / tot, 4) if tot else None
    per, frames_matched = (frame_counters(prof, kname, args.warmup, steps) if prof is not None and match
                           else ({}, False))
    if per:
        line["profile_frames_matched"] = frames_matched
        hbm = per.get("hbm_bytes")
        line["traffic"] = int(hbm) if hbm else None
        if per.get("GRBM_GUI_ACTIVE") and per.get("duration_ns"):
            line["pmc_clock_ghz"] = round(per["GRBM_GUI_ACTIVE"] / 8.0 / per["duration_ns"], 3)
            line["pmc_kernel_ms"] = round(per["duration_ns"] * 1e-6, 4)
        valu = per.get("SQ_INSTS_VALU", 0.0)
        mf = per.get("SQ_INSTS_MFMA", 0.0)
        mfb = per.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
        if valu:
            line["valu_insts_per_step"] = valu
            line["valu_insts_per_cast"] = round(valu / casts_per_frame, 2)
            line["valu_issue_frac"] = round(valu / t / 1e9 / VALU_ISSUE_PEAK_G, 4)
        if mf:
            line["mfma_insts_per_step"] = mf
            line["mfma_insts_per_cast"] = round(mf / casts_per_frame, 3)
        if mfb:
            line["mfma_busy_frac"] = round(mfb / (1024 * 2.4e9 * t), 4)
        if per.get("SQ_WAVE_CYCLES") and per.get("SQ_WAIT_ANY") is not None:
            line["wave_cycles_waiting_frac"] = round(per["SQ_WAIT_ANY"] / per["SQ_WAVE_CYCLES"], 4)
            if per.get("SQ_ACTIVE_INST_ANY"):
                line["wave_cycles_issuing_frac"] = round(per["SQ_ACTIVE_INST_ANY"] / per["SQ_WAVE_CYCLES"], 4)
        if bound == "valu" and valu:
            line["achieved"] = round(valu / t / 1e9, 1)
            line["frac"] = round(line["achieved"] / VALU_ISSUE_PEAK_G, 4)
            if line.get("pmc_clock_ghz"):
                line["frac_at_pmc_clock"] = round(valu / (1024 * line["pmc_clock_ghz"] * 1e9 * t / 2.0), 4)
        bf16 = per.get("SQ_INSTS_VALU_MFMA_BF16", 0.0)
        if bound == "mfma" and bf16:
            line["executed_bf16_tflops"] = round(bf16 * 16384 / t / 1e12, 1)  # 16x16x32 bf16
            line["executed_frac"] = round(line["executed_bf16_tflops"] / MFMA_BF16_PEAK_TFLOPS, 4)
    if per and line["traffic"]:
        # the HBM leg of the same kernel: measured DRAM bytes per frame / its time
        line["hbm_gbs"] = round(line["traffic"] / t / 1e9, 1)
        line["hbm_frac"] = round(line["hbm_gbs"] / HBM_PEAK_GBS, 4)
        if prof.get("fetch_scale") == 1:
            line["traffic_note"] = ("FETCH_SIZE + WRITE_SIZE at the L2's fabric side, FETCH_SIZE not doubled "
                                    "(gathers, not 16-B streams); Infinity-Cache hits included, so an upper "
                                    "bound on DRAM bytes")
    line["kernels"] = kernel_table(prof if match else None, args, kt)
    # what the counters say holds the kernel back: the busiest pipe, or latency when no pipe
    # is near its roof and most wave cycles wait (s_waitcnt / barrier)
    pipes = {"valu_issue": line.get("valu_issue_frac"), "hbm": line.get("hbm_frac"),
             "matrix": line.get("mfma_busy_frac")}
    pipes = {k: v for k, v in pipes.items() if v is not None}
    wait = line.get("wave_cycles_waiting_frac")
    if pipes:
        top = max(pipes, key=pipes.get)
        if wait is not None and wait > 0.4 and pipes[top] < 0.5:
            line["limiter"] = (f"latency: {wait:.0%} of wave cycles waiting on memory / LDS, busiest pipe "
                               f"{top} at {pipes[top]:.0%}")
        else:
            line["limiter"] = f"{top} at {pipes[top]:.0%}"
    if bound == "mfma":
        n_in = geom.nn_vertices.size
        dims = [n_in, 200, 300, 200, 144]
        flop_ray = 2 * sum(dims[i] * dims[i + 1] for i in range(4))
        rows = casts_per_frame - params.width * params.height * params.spp  # bounce casts = forwards
        line["reference_flops_per_ray"] = flop_ray
        line["forwards_per_step"] = int(rows)
        line["reference_algorithmic_tflops"] = round(rows * flop_ray / t / 1e12, 1)
        line["reference_algorithmic_frac"] = round(line["reference_algorithmic_tflops"] / MFMA_BF16_PEAK_TFLOPS, 4)
        # the roofline proper: what the matrix cores executed (None without a matching profile)
        line["achieved"] = line.get("executed_bf16_tflops")
        line["frac"] = line.get("executed_frac")
    else:
        if line.get("hbm_frac") is not None and line["frac"] is not None and line["hbm_frac"] > line["frac"]:
            # more of the HBM roof than of the VALU issue roof is in use: HBM bounds it
            line.update({"bound": "hbm", "achieved": line["hbm_gbs"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": line["hbm_frac"], "valu_frac": line["frac"]})
        n_tri = geom.n_tri
        useful = casts_per_frame * 71.0 * n_tri / t / 1e12
        line["brute_force_tflops"] = round(useful, 2)
        line["brute_force_frac_of_fp32"] = round(useful / VALU_PEAK_TFLOPS, 4)
        b_cast = 36 * n_tri + 32
        line["hbm_algorithmic_bytes_per_cast"] = b_cast
        line["hbm_algorithmic_ratio"] = round(casts_per_frame * b_cast / t / 1e9 / HBM_PEAK_GBS, 3)
    return line


def kernel_table(prof, args, kt: dict) -> dict:
    """Every timed kernel family of the frame: its time per step (HIP events) and share, and
    from the build's profile (when it matches) its VALU issue, matrix-pipe and HBM fractions
    over that time -- e.g. the DQN frame's k_dqn_bounce beside the k_dqn_mlp roofline."""
    steps = args.steps
    tot = sum(v[0] for v in kt.values()) or 1.0
    out = {}
    for fam, (ms, n) in kt.items():
        if not n:
            continue
        name = rtmi.ktime_name(fam)
        t = ms / steps * 1e-3
        e = {"ms_per_step": round(t * 1e3, 4), "launches_per_step": n / steps, "share": round(ms / tot, 4)}
        if prof is not None:
            per, _ = frame_counters(prof, name + "<", args.warmup, steps)
            if per.get("SQ_INSTS_VALU"):
                e["valu_issue_frac"] = round(per["SQ_INSTS_VALU"] / t / 1e9 / VALU_ISSUE_PEAK_G, 4)
            if per.get("SQ_VALU_MFMA_BUSY_CYCLES"):
                e["mfma_busy_frac"] = round(per["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * 2.4e9 * t), 4)
            if per.get("hbm_bytes"):
                e["hbm_bytes_per_step"] = int(per["hbm_bytes"])
                e["hbm_frac"] = round(per["hbm_bytes"] / t / 1e9 / HBM_PEAK_GBS, 4)
        out[name] = e
    return out


def progress(msg: str) -> None:
    """a stderr line per stage (long runs stay visibly alive; stdout keeps the one JSON line)"""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def cpu_baseline_learned(sampler, geom, params, cam_pos, seconds, q_state=None, frame_index=0):
    """The CPU restatement (oracle/, OpenMP over rows) on a bounded sample of a learned-sampler
    frame, best of 3 ("for configs 4-5, CPU time may be measured on a reduced
    SPP"; a sample's cost does not depend on the frame's spp).
    sarsa: rows of the 512^2 door_room frame (the restatement's Expected SARSA: the KD search,
      the CDF sampling, the TD accumulation), 16 spp per pixel, from the Q-table the GPU map
      held at the first timed frame (q_state: the same frame index as the GPU's timed frames);
    dqn: a 64^2 window at the frame's centre with the bf16-emulating forward of the same
      synthetic weights at every bounce (oracle.render_dqn), spp from the time budget."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # test infrastructure: the CPU baseline leg only

    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or os.cpu_count() or 1
    oracle.set_threads(threads)
    ocam = oracle.camera(cam_pos)
    W, H = params.width, params.height
    if sampler == "sarsa":
        m = oracle.Sarsa(geom, int(params.seed))
        if q_state is not None:
            m.load_q(q_state)
        sp = rtmi.default_params(params.preset, width=W, height=H, spp=16, spp_split=1)
        op = oracle.params_from(sp)
        rows = max(16, threads)
        t0 = time.perf_counter()
        _, casts = m.render_rect(ocam, op, (0, H // 2 - rows // 2, W, rows))
        rate = casts / max(time.perf_counter() - t0, 1e-9)
        rows = int(max(rows, min(H, seconds * rate / max(casts / rows, 1.0))))
        rect = (0, max(0, H // 2 - rows // 2), W, rows)
        run = lambda: m.render_rect(ocam, op, rect)  # noqa: E731
        state = (f"frame {frame_index} (the Q-table of the GPU map at the first timed frame, loaded into the "
                 f"restatement)" if q_state is not None else "frame 0")
        what = (f"rows {rect[1]}..{rect[1] + rows - 1} of {state} of the {W}x{H} Expected-SARSA frame at 16 spp "
                f"per pixel (the frame's own spp {params.spp}: per-sample cost is independent of it)")
    else:
        Ws, bs = rtmi.dqn.synthetic_weights(geom.nn_vertices.size)
        win = 64
        rect = (W // 2 - win // 2, H // 2 - win // 2, win, win)
        op1 = oracle.params_from(rtmi.default_params(params.preset, width=W, height=H, spp=1))
        t0 = time.perf_counter()
        _, casts = oracle.render_dqn(geom, Ws, bs, geom.nn_vertices, ocam, op1, rect, bf16=True)
        dt = time.perf_counter() - t0
        spp = int(max(1, min(params.spp, seconds / max(dt, 1e-9))))
        op = oracle.params_from(rtmi.default_params(params.preset, width=W, height=H, spp=spp))
        run = lambda: oracle.render_dqn(geom, Ws, bs, geom.nn_vertices, ocam, op, rect, bf16=True)  # noqa: E731
        what = (f"the {win}x{win} window at ({rect[0]}, {rect[1]}) of the {W}x{H} frame at {spp} spp, "
                f"bf16-emulating DQN forward at every bounce (the frame's own spp {params.spp}: per-sample "
                f"cost is independent of it)")
    best, casts = None, 0
    for i in range(3):
        t0 = time.perf_counter()
        _, casts = run()
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
        progress(f"cpu baseline run {i + 1}/3: {casts} ray casts in {dt:.2f} s")
    return {"value": round(casts / best / 1e6, 3), "unit": "Mrays/s", "cores": threads, "kind": "port",
            "sample": f"{what}; {casts} ray casts, best of 3: {best:.2f} s, OpenMP over rows"}


def cpu_baseline(geom, params, cam_pos, seconds):
    """Time the CPU restatement (oracle/, OpenMP over rows) on a bounded strip of the same frame,
    best of 3, and one thread on a 2-row strip.  A frame whose rows cost
    more than the budget is sampled at fewer spp (<= 16 per pixel: a sample's cost does not
    depend on the frame's spp); the strip is then not the frame's own pixels (no parity strip)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # test infrastructure: the CPU baseline leg only

    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or os.cpu_count() or 1
    oracle.set_threads(threads)
    ocam = oracle.camera(cam_pos)
    w = params.width
    sp = params
    if params.spp > 16:
        sp = rtmi.default_params(params.preset, width=params.width, height=params.height, spp=16,
                                 spp_split=min(params.spp_split, 16))
    op = oracle.params_from(sp)
    rows, y0 = max(4, min(threads, 16)), params.height // 2 - 2
    t0 = time.perf_counter()
    _, casts = oracle.render(geom, ocam, op, (0, y0, w, rows))
    rate = casts / max(time.perf_counter() - t0, 1e-9)
    per_row = casts / rows
    if sp is not params and rate * seconds >= per_row * params.spp / sp.spp * params.height:
        sp, op = params, oracle.params_from(params)  # the whole frame at its own spp fits the budget
        per_row *= params.spp / 16
    rows = int(max(4, min(params.height, seconds * rate / max(per_row, 1.0))))
    if rows >= 0.6 * params.height:  # most of the frame anyway: take all of it (a full-frame parity check)
        rows = params.height
    y0 = max(0, params.height // 2 - rows // 2)
    best, strip = None, None
    for i in range(3):
        t0 = time.perf_counter()
        strip, casts = oracle.render(geom, ocam, op, (0, y0, w, rows))
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
        progress(f"cpu baseline run {i + 1}/3: rows {y0}..{y0 + rows - 1} at {sp.spp} spp, {casts} ray casts in {dt:.2f} s")
    oracle.set_threads(1)
    y1 = params.height // 2 - 1
    t0 = time.perf_counter()
    _, casts1 = oracle.render(geom, ocam, op, (0, y1, w, 2))
    dt1 = time.perf_counter() - t0
    oracle.set_threads(threads)
    own = sp is params
    return {
        "value": round(casts / best / 1e6, 3),
        "unit": "Mrays/s",
        "cores": threads,
        "kind": "port",
        "sample": f"rows {y0}..{y0 + rows - 1} of the {w}x{params.height} frame at {sp.spp} spp"
                  + ("" if own else f" (the frame's own spp {params.spp}: per-sample cost is independent of it)")
                  + f" ({casts} ray casts, best of 3: {best:.2f} s, OpenMP over rows)",
        "value_1thread": round(casts1 / max(dt1, 1e-9) / 1e6, 3),
        "sample_1thread": f"rows {y1}..{y1 + 1} at {sp.spp} spp ({casts1} ray casts, {dt1:.2f} s, 1 thread)",
    }, ((y0, rows, strip, casts) if own else None)


def parity_strip(ctx, scene, cam, params, image, strip_run):
    """The CPU baseline's own render (rows y0..y0+rows-1, the whole frame when the time budget
    allows) against the same rows of the GPU frame: bits, MAPE, and the ray casts of a
    separate GPU render of the strip.  No extra CPU work."""
    y0, rows, ref, ref_casts = strip_run
    got = image[y0:y0 + rows]
    _, gpu_casts = rtmi.render(ctx, scene, cam, params, (0, y0, params.width, rows))
    return {"rows": [y0, y0 + rows - 1], "pixels": int(rows * params.width),
            "frac_of_frame": round(rows / params.height, 4),
            "mape_vs_cpu": rtmi.metrics.mape_f(ref, got),
            "bit_exact": bool(np.array_equal(ref.view(np.uint32), got.view(np.uint32))),
            "ray_casts_equal": gpu_casts == ref_casts, "ray_casts": int(ref_casts)}


def parity_tiles(ctx, scene, geom, params, cam, cam_pos, image):
    """8 full 32x32 tiles spread over the frame: the frame's pixels bit-exact vs the CPU
    restatement, and the tile's ray casts (a separate GPU render of the tile) equal to its."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle

    op = oracle.params_from(params)
    ocam = oracle.camera(cam_pos)
    W, H = params.width, params.height
    fx = [0.08, 0.45, 0.8, 0.25, 0.6, 0.92, 0.1, 0.5]
    fy = [0.1, 0.15, 0.3, 0.45, 0.55, 0.7, 0.85, 0.95]
    worst, exact, casts_ok, px = 0.0, True, True, 0
    for a, b in zip(fx, fy):
        x = min(W - TILE, int(a * W) // TILE * TILE)
        y = min(H - TILE, int(b * H) // TILE * TILE)
        ref, ref_casts = oracle.render(geom, ocam, op, (x, y, TILE, TILE))
        got = image[y:y + TILE, x:x + TILE]
        _, gpu_casts = rtmi.render(ctx, scene, cam, params, (x, y, TILE, TILE))
        worst = max(worst, rtmi.metrics.mape_f(ref, got))
        exact = exact and bool(np.array_equal(ref.view(np.uint32), got.view(np.uint32)))
        casts_ok = casts_ok and gpu_casts == ref_casts
        px += TILE * TILE
    return {"mape_vs_cpu": worst, "bit_exact": exact, "ray_casts_equal": casts_ok, "tiles": len(fx),
            "pixels": px, "frac_of_frame": round(px / (W * H), 4)}


def make_workload(args, ctx):
    scene_kind, preset, sampler, W, H, spp, split, cfg = WORKLOADS[args.workload]
    W = args.width or W
    H = args.height or H
    spp = args.spp or spp
    split = args.spp_split or split
    if scene_kind == "cornell":
        geom = rtmi.cornell_geometry(preset)
        cam_pos = rtmi.CAMERAS["cornell"]
    else:
        geom = rtmi.obj_geometry(os.path.join(MODELS, scene_kind + ".obj"), scene_kind)
        cam_pos = rtmi.CAMERAS[scene_kind]
    params = rtmi.default_params(preset, width=W, height=H, spp=spp, spp_split=split)
    if args.workload == "cornell" and (W, H, spp) == (256, 256, 4):
        cfg = 1  # BASELINE config 1: the reference's CPU-runnable Cornell case
    return scene_kind, sampler, cfg, geom, cam_pos, params


class _LocalGather:
    """Stand-in for the RCCL gather in a one-GPU emulation of rank r of P: the rank's tile
    buffer is copied into its slot of a [P, k, T, T, 3] buffer on a second stream, ordered
    after the render the way the collective is (the next render into the buffer waits for it)."""

    def __init__(self, world: int, shape, device, rank: int):
        self.stream = torch.cuda.Stream(device)
        self.buf = torch.empty((world,) + tuple(shape), dtype=torch.float32, device=device)
        self.rank = rank
        self.done = [None, None]

    def gather(self, out: torch.Tensor, b: int) -> None:
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(out.device))
        with torch.cuda.stream(self.stream):
            self.stream.wait_event(ev)
            self.buf[self.rank].copy_(out, non_blocking=True)
            self.done[b] = torch.cuda.Event()
            self.done[b].record(self.stream)

    def wait(self, b: int) -> None:
        if self.done[b] is not None:
            torch.cuda.current_stream().wait_event(self.done[b])
            self.done[b] = None


def emulate(args) -> None:
    """--emulate-ranks P: the P-GPU step predicted on one GPU.  For every rank r of P, its tile
    set (rtmi.tiles.rank_tiles: the tiles it renders at world size P) runs through the same timed
    loop as a real rank -- warmup, then `steps` frames, each: wait for the buffer's previous
    gather, record events, render (the ctypes call and its launches), queue the gather -- with a
    device copy on a second stream standing in for the RCCL gather to rank 0.  The P-GPU step is
    the slowest rank's host-inclusive step time; the one-GPU step is the same loop over all tiles.
    Expected SARSA adds its real exchange: the TD sums' all-reduce, whose payload is reported with
    a ring-all-reduce model over one xGMI link (it cannot run on one GPU)."""
    P = args.emulate_ranks
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    ctx = rtmi.Context(0)
    scene_kind, sampler, cfg, geom, cam_pos, params = make_workload(args, ctx)
    scene = rtmi.Scene(ctx, geom)
    cam = rtmi.camera(cam_pos)
    stream = torch.cuda.current_stream(dev)
    casts = torch.zeros(1, dtype=torch.int64, device=dev)
    extra = []
    rmap = None
    if sampler == "sarsa":
        rmap = rtmi.sarsa.RadianceMap(ctx, scene, 1984)
        extra.append(rmap)
    elif sampler == "dqn":
        Ws, bs = rtmi.dqn.synthetic_weights(geom.nn_vertices.size)
        net = rtmi.dqn.Dqn(ctx, geom.nn_vertices, Ws, bs)
        extra.append(net)

    def make_render(tiles, n_real, world):
        if sampler == "sarsa":
            def render(out):
                # every timed frame (one GPU and each rank alike) reads the map as the shared
                # warmup left it and leaves its TD sums unapplied, as a rank's frame leaves them
                # for the exchange: the ranks' frames are the same frame of the same learning run
                rmap.render_tiles_device(cam, params, tiles[:n_real], TILE, out.data_ptr(), casts.data_ptr(),
                                         apply=False, stream=stream.cuda_stream)
        elif sampler == "dqn":
            def render(out):
                rtmi.dqn.render_tiles_device(ctx, scene, net, cam, params, tiles, TILE, out.data_ptr(),
                                             casts.data_ptr(), stream.cuda_stream)
        else:
            def render(out):
                rtmi.render_tiles_device(ctx, scene, cam, params, tiles, TILE, out.data_ptr(), casts.data_ptr(),
                                         stream.cuda_stream)
        return render

    if sampler == "sarsa":  # the learning run's warmup frames, once, on the whole frame
        wt = rtmi.tiles.rank_tiles(params.width, params.height, TILE, 0, 1)
        wo = torch.zeros((wt.shape[0], TILE, TILE, 3), dtype=torch.float32, device=dev)
        for _ in range(args.warmup):
            rmap.render_tiles_device(cam, params, wt, TILE, wo.data_ptr(), casts.data_ptr(), apply=True,
                                     stream=stream.cuda_stream)
        torch.cuda.synchronize()

    def run(world, rank):
        tiles = rtmi.tiles.rank_tiles(params.width, params.height, TILE, rank, world)
        n_real = rtmi.tiles.rank_tile_count(params.width, params.height, TILE, rank, world)
        shape = (tiles.shape[0], TILE, TILE, 3)
        render = make_render(tiles, n_real, world)
        outs = [torch.zeros(shape, dtype=torch.float32, device=dev) for _ in range(2)]
        g = _LocalGather(world, shape, dev, rank)
        for i in range(args.warmup):
            g.wait(i % 2)
            render(outs[i % 2])
            g.gather(outs[i % 2], i % 2)
        torch.cuda.synchronize()
        casts.zero_()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(args.steps):
            b = i % 2
            g.wait(b)
            ev[i][0].record(stream)
            render(outs[b])
            ev[i][1].record(stream)
            g.gather(outs[b], b)
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
        kern = float(np.mean([a.elapsed_time(b) for a, b in ev]))
        return {"rank": rank, "tiles": int(n_real), "ms_per_step": round(elapsed / args.steps * 1e3, 4),
                "frame_ms": round(kern, 4), "host_ms_over_device": round(elapsed / args.steps * 1e3 - kern, 4),
                "ray_casts_per_step": int(casts.item()) // args.steps}

    progress(f"{args.workload}: one GPU, all tiles")
    one = run(1, 0)
    ranks = []
    for r in range(P):
        ranks.append(run(P, r))
        progress(f"rank {r} of {P}: {ranks[-1]['ms_per_step']} ms per step")
    t_p = max(x["ms_per_step"] for x in ranks)
    line = {"mode": "emulated_ranks", "workload": args.workload, "baseline_config": cfg, "emulated_world": P,
            "width": params.width, "height": params.height, "spp": params.spp, "steps": args.steps,
            "warmup": args.warmup, "one_gpu": one, "ranks": ranks,
            "predicted_step_ms": t_p,
            "predicted_speedup": round(one["ms_per_step"] / t_p, 3),
            "predicted_speedup_device_only": round(one["frame_ms"] / max(x["frame_ms"] for x in ranks), 3),
            "gather_bytes_per_rank": int(rtmi.tiles.rank_tiles(params.width, params.height, TILE, 0, P).shape[0]
                                         * TILE * TILE * 12)}
    if sampler == "sarsa":
        # the frame's update (k_sarsa_apply over the whole map) runs on every rank after the
        # exchange, at any P: timed here on its own, added to both sides
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            rmap.apply(stream.cuda_stream)
        torch.cuda.synchronize()
        apply_ms = (time.perf_counter() - t0) / args.steps * 1e3
        n = rmap.n_volumes * 144
        payload = n * (8 + 4)  # int64 sums + int32 counts
        ring = 2.0 * (P - 1) / P * payload / 153e9 * 1e3  # ms over one 153 GB/s xGMI link
        line["apply_ms"] = round(apply_ms, 4)
        line["td_allreduce_bytes"] = payload
        line["td_allreduce_ms_model"] = round(ring, 3)
        one_step = one["ms_per_step"] + apply_ms
        p_step = t_p + ring + apply_ms
        line["one_gpu_step_ms_with_apply"] = round(one_step, 4)
        line["predicted_step_ms_with_apply_and_allreduce_model"] = round(p_step, 4)
        line["predicted_speedup_with_apply_and_allreduce_model"] = round(one_step / p_step, 3)
    print(json.dumps(line), flush=True)
    for o in extra:
        o.close()
    scene.close()
    ctx.close()


def main():
    args = parse()
    if args.emulate_ranks > 1:
        return emulate(args)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:  # (rank_launch refuses this before any GPU work; kept for imports of main)
        raise SystemExit(f"WORLD_SIZE={world} but --gpus {args.gpus}")
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # the rank's GPU first, then the process group bound to it (RCCL's communicator is created on
    # that device, not on whichever device is current when the first collective runs)
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if world > 1:
        dist.init_process_group(backend="nccl", device_id=dev)

    ctx = rtmi.Context(local_rank)
    scene_kind, sampler, cfg, geom, cam_pos, params = make_workload(args, ctx)
    scene = rtmi.Scene(ctx, geom)
    cam = rtmi.camera(cam_pos)

    tiles = rtmi.tiles.rank_tiles(params.width, params.height, TILE, rank, world)
    n_real = rtmi.tiles.rank_tile_count(params.width, params.height, TILE, rank, world)
    k = tiles.shape[0]
    casts = torch.zeros(1, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream(dev)
    extra = []  # objects to close

    if sampler == "sarsa":
        rmap = rtmi.sarsa.RadianceMap(ctx, scene, 1984)
        extra.append(rmap)
        td = rtmi.dist.td_tensors(rmap, dev) if world > 1 else None

        def render(out):
            rtmi.dist.sarsa_frame(rmap, cam, params, tiles, n_real, TILE, out, casts, td)
    elif sampler == "dqn":
        Ws, bs = rtmi.dqn.synthetic_weights(geom.nn_vertices.size)
        net = rtmi.dqn.Dqn(ctx, geom.nn_vertices, Ws, bs)
        extra.append(net)

        def render(out):
            rtmi.dqn.render_tiles_device(ctx, scene, net, cam, params, tiles, TILE, out.data_ptr(),
                                         casts.data_ptr(), stream.cuda_stream)
    else:
        def render(out):
            rtmi.render_tiles_device(ctx, scene, cam, params, tiles, TILE, out.data_ptr(), casts.data_ptr(),
                                     stream.cuda_stream)

    # two frame buffers: frame i+1 renders while frame i is gathered to rank 0 over RCCL
    pipe = rtmi.dist.FramePipeline(render, (k, TILE, TILE, 3), world, dev)
    for i in range(args.warmup):
        pipe.gather_frame(pipe.render_frame(i))
    pipe.drain()
    q_state = None
    if sampler == "sarsa" and rank == 0 and args.cpu_seconds > 0 and world == 1:
        q_state = rmap.read()[0]  # (before the timed region) the CPU baseline's starting Q-table
    if rank == 0:
        progress(f"{args.workload}: {args.warmup} warmup frame(s) done, timing {args.steps}")
    torch.cuda.synchronize()
    casts.zero_()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    rtmi.ktime_enable(True)  # the kernels' own launches, HIP events on their launch stream
    t0 = time.perf_counter()
    for i in range(args.steps):
        pipe.wait(i % 2)  # outside the kernel's event window
        ev[i][0].record(stream)
        b = pipe.render_frame(i)
        ev[i][1].record(stream)
        pipe.gather_frame(b)
    pipe.drain()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kt = rtmi.ktime_read()
    rtmi.ktime_enable(False)

    frame_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    rank_casts = int(casts.item())
    if world > 1:
        t_max = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t_max, op=dist.ReduceOp.MAX)
        tot = torch.tensor([rank_casts], dtype=torch.int64, device=dev)
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
        elapsed, total_casts = float(t_max.item()), int(tot.item())
    else:
        total_casts = rank_casts

    frame = pipe.frame(args.steps - 1)
    if rank == 0:
        progress(f"timed: {elapsed / args.steps * 1e3:.3f} ms per step")
        image = rtmi.tiles.assemble(frame.cpu().numpy(), params.width, params.height, TILE, world)
        line = {
            "metric": f"Mrays/sec ({WORKLOADS[args.workload][0]} {params.width}^2 {params.spp}spp ray casts)"
            if params.width == params.height else f"Mrays/sec ({args.workload} ray casts)",
            "value": round(total_casts / elapsed / 1e6, 2),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": ("procedural Cornell box of the reference (CPU-engine preset)" if scene_kind == "cornell"
                     else f"Models/{scene_kind}.obj of the reference (GPU-engine preset)")
            + ", Philox RNG seed 1984" + (", synthetic He-normal DQN weights" if sampler == "dqn" else ""),
            "config": {
                "workload": f"{scene_kind}_{params.width}x{params.height}_{params.spp}spp"
                + ("" if sampler == "uniform" else f"_{sampler}"),
                "baseline_config": cfg,
                "width": params.width, "height": params.height, "spp": params.spp,
                "max_bounces": params.max_bounces,
                "hit_rule": "cpu_object" if params.hit_rule == rtmi.RT_HIT_RULE_CPU else "gpu_engine",
                "sampler": sampler, "spp_split": params.spp_split, "tile": TILE, "parallelism": f"tiles{world}",
                "triangles": geom.n_tri,
            },
            "ray_casts_per_step": total_casts // args.steps,
            "frame_ms": round(frame_ms, 4),
            "roofline": roofline(args, geom, params, rank_casts / args.steps, kt),
        }
        # preprocessing outside the timed region, measured in this run: the scene's bounce-ray
        # candidate table (host build + upload on the first render that takes it, like a BVH
        # build; device bytes per rank).  The camera rays' cull runs inside every timed frame.
        tab_rule = rtmi.RT_HIT_RULE_GPU if sampler == "dqn" else params.hit_rule
        ti = scene.ctab_info(tab_rule)
        line["config"]["candidate_table"] = {
            "built": ti["built"], "hit_rule": "cpu_object" if tab_rule == rtmi.RT_HIT_RULE_CPU else "gpu_engine",
            "table_build_s": round(ti["build_s"], 3), "table_bytes": ti["bytes"],
            "camera_ray_cull": "in the timed frame"}
        if sampler == "sarsa":  # a learning run: which of its frames the line times
            line["config"]["frames_warmup"] = [0, args.warmup - 1] if args.warmup else []
            line["config"]["frames_timed"] = [args.warmup, args.warmup + args.steps - 1]
        if sampler == "uniform" and not args.no_parity and params.width % TILE == 0 and params.height % TILE == 0:
            line["parity"] = parity_tiles(ctx, scene, geom, params, cam, cam_pos, image)
        if args.cpu_seconds > 0 and world == 1:  # the CPU baseline is an N=1 figure
            if sampler == "uniform":
                line["cpu_baseline"], strip_run = cpu_baseline(geom, params, cam_pos, args.cpu_seconds)
                if "parity" in line and strip_run is not None:  # the baseline's strip is the same frame: check it too
                    line["parity"]["cpu_strip"] = parity_strip(ctx, scene, cam, params, image, strip_run)
            else:
                line["cpu_baseline"] = cpu_baseline_learned(sampler, geom, params, cam_pos, args.cpu_seconds,
                                                            q_state, args.warmup)
        print(json.dumps(line), flush=True)

    for o in extra:
        o.close()
    scene.close()
    ctx.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
