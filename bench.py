#!/usr/bin/env python3
"""Benchmark: Mrays/s on the Cornell box 512x512, 256 spp (BASELINE.json config 2).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

A step renders one full 512x512 / 256-spp frame of the reference's Cornell
box (CPU-engine preset: cap 2 bounces, hit rule of the prebuilt CPU object,
uniform hemisphere sampling).  The frame is cut into 32x32 tiles dealt to the
ranks by diagonals (rtmi.tiles; one process per GPU); each rank renders its
tiles with the HIP megakernel, and the per-rank tile buffers are all-gathered
over RCCL into the full image -- asynchronously, into one of two buffers, so
frame i+1 renders while frame i is exchanged.  The frame is fixed as N grows:
strong scaling.

value = total ray casts (all ranks) / max-over-ranks wall time of the K
timed steps, in Mrays/s.  rank 0 prints one JSON line with the roofline of
the render kernel (HIP events on the launch stream), the per-pixel MAPE vs the
CPU restatement on a checked window, and the CPU baseline (oracle/, timed on
this host's cores on a bounded sample).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "reinforcement-light-rays-pathtracer_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import rtmi  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
VALU_PEAK_TFLOPS = 157.3  # FP32 vector spec
TILE = 32
# HBM traffic of k_render<0,0,0> on this workload from the PMC passes of tools/gpu_profile.sh
# (rocprofv3 FETCH_SIZE x 2 per MI355X_MICROARCH.md + WRITE_SIZE, per launch)
PMC_PROFILE = os.path.join("profiles", "r1v9_pmc.json")
DEFAULT_WORKLOAD = (512, 512, 256, 64)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--width", type=int, default=512)
    ap.add_argument("--height", type=int, default=512)
    ap.add_argument("--spp", type=int, default=256)
    ap.add_argument("--spp-split", type=int, default=64)
    ap.add_argument("--cpu-seconds", type=float, default=12.0,
                    help="target CPU-baseline sample duration (0 disables)")
    ap.add_argument("--no-parity", action="store_true")
    return ap.parse_args()


def pmc_traffic(params):
    """(bytes per launch, source) of the committed PMC profile for the default workload."""
    if (params.width, params.height, params.spp, params.spp_split) != DEFAULT_WORKLOAD:
        return None, None
    try:
        prof = json.load(open(os.path.join(ROOT, PMC_PROFILE)))
    except (OSError, ValueError):
        return None, None
    for name, e in prof.get("selected", {}).items():
        if "k_render<0, 0, 0" in name and "traffic_bytes_per_launch" in e:
            return int(e["traffic_bytes_per_launch"]), PMC_PROFILE
    return None, None


SQ_PROFILE = os.path.join("profiles", "r1v9_sq_summary.json")


def pmc_valu_issue(params):
    """Fraction of the VALU issue slots k_render used on this workload (SQ_INSTS_VALU of
    the committed PMC pass over 1024 SIMDs x one wave-instruction per 2 cycles)."""
    if (params.width, params.height, params.spp, params.spp_split) != DEFAULT_WORKLOAD:
        return None
    try:
        c = json.load(open(os.path.join(ROOT, SQ_PROFILE)))["per_dispatch"]
        cycles = c["GRBM_GUI_ACTIVE"] / 8.0  # summed over the 8 XCDs
        return round(c["SQ_INSTS_VALU"] / (1024 * cycles / 2.0), 3)
    except (OSError, ValueError, KeyError):
        return None


def cpu_baseline(geom, params, cam_pos, seconds):
    """Time the CPU restatement (oracle/, OpenMP) on a bounded strip of the same frame."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # test infrastructure: the CPU baseline leg only

    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or os.cpu_count() or 1
    oracle.set_threads(threads)
    op = oracle.params_from(params)
    ocam = oracle.camera(cam_pos)
    w = params.width
    rows, y0 = 4, params.height // 2 - 2
    t0 = time.perf_counter()
    _, casts = oracle.render(geom, ocam, op, (0, y0, w, rows))
    dt = time.perf_counter() - t0
    rate = casts / max(dt, 1e-9)
    # scale the strip so that the timed sample takes about `seconds`
    per_row = casts / rows
    rows = int(max(4, min(params.height, seconds * rate / max(per_row, 1.0))))
    y0 = max(0, params.height // 2 - rows // 2)
    best = None
    for _ in range(1):
        t0 = time.perf_counter()
        _, casts = oracle.render(geom, ocam, op, (0, y0, w, rows))
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
    # the 1-thread figure on a 2-row strip of the same frame
    oracle.set_threads(1)
    y1 = params.height // 2 - 1
    t0 = time.perf_counter()
    _, casts1 = oracle.render(geom, ocam, op, (0, y1, w, 2))
    dt1 = time.perf_counter() - t0
    oracle.set_threads(threads)
    return {
        "value": round(casts / best / 1e6, 3),
        "unit": "Mrays/s",
        "cores": threads,
        "kind": "port",
        "sample": f"rows {y0}..{y0 + rows - 1} of the {w}x{params.height}/{params.spp}-spp frame "
                  f"({casts} ray casts, {best:.1f} s, OpenMP over rows)",
        "value_1thread": round(casts1 / max(dt1, 1e-9) / 1e6, 3),
        "sample_1thread": f"rows {y1}..{y1 + 1} ({casts1} ray casts, {dt1:.2f} s, 1 thread)",
    }


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group(backend="nccl")
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)

    ctx = rtmi.Context(local_rank)
    geom = rtmi.cornell_geometry(rtmi.RT_PRESET_CPU)
    scene = rtmi.Scene(ctx, geom)
    params = rtmi.default_params(rtmi.RT_PRESET_CPU, width=args.width, height=args.height,
                                 spp=args.spp, spp_split=args.spp_split)
    cam_pos = rtmi.CAMERAS["cornell"]
    cam = rtmi.camera(cam_pos)

    tiles = rtmi.tiles.rank_tiles(params.width, params.height, TILE, rank, world)
    k = tiles.shape[0]
    casts = torch.zeros(1, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream(dev)

    def render(out):
        rtmi.render_tiles_device(ctx, scene, cam, params, tiles, TILE, out.data_ptr(), casts.data_ptr(),
                                 stream.cuda_stream)

    # two frame buffers: frame i+1 renders while frame i is all-gathered over RCCL
    pipe = rtmi.dist.FramePipeline(render, (k, TILE, TILE, 3), world, dev)
    for i in range(args.warmup):
        pipe.gather_frame(pipe.render_frame(i))
    pipe.drain()
    torch.cuda.synchronize()
    casts.zero_()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
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

    kernel_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    rank_casts = int(casts.item())
    stats = torch.tensor([elapsed, float(rank_casts), kernel_ms, float(rank_casts)],
                         dtype=torch.float64, device=dev)
    if world > 1:
        t_max = stats[0:1].clone()
        dist.all_reduce(t_max, op=dist.ReduceOp.MAX)
        tot = stats[1:2].clone()
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
        elapsed, total_casts = float(t_max.item()), int(tot.item())
    else:
        total_casts = rank_casts

    frame = pipe.frame(args.steps - 1)
    image = None
    if rank == 0:
        image = rtmi.tiles.assemble(frame.cpu().numpy(), params.width, params.height, TILE, world)

    if rank == 0:
        n_tri = geom.n_tri
        b_cast = 36 * n_tri + 32  # algorithmic bytes per ray cast
        casts_per_launch = rank_casts / args.steps
        achieved_gbs = casts_per_launch * b_cast / (kernel_ms * 1e-3) / 1e9
        valu_tflops = casts_per_launch * n_tri * 71 / (kernel_ms * 1e-3) / 1e12
        traffic, traffic_src = pmc_traffic(params)
        line = {
            "metric": "Mrays/sec (Cornell 512^2 256spp ray casts)",
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
            "data": "procedural Cornell box of the reference (CPU-engine preset), Philox RNG seed 1984",
            "config": {
                "workload": "cornell_512x512_256spp",
                "width": params.width, "height": params.height, "spp": params.spp,
                "max_bounces": params.max_bounces, "hit_rule": "cpu_object", "sampler": "uniform",
                "spp_split": params.spp_split, "tile": TILE, "parallelism": f"tiles{world}",
                "triangles": n_tri,
            },
            "ray_casts_per_step": total_casts // args.steps,
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved_gbs, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved_gbs / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "traffic_source": traffic_src,
                "kernel": "k_render<0,0,0>",
                "kernel_ms": round(kernel_ms, 4),
                "bytes_per_cast": b_cast,
                "valu_tflops_est": round(valu_tflops, 2),
                "valu_frac_est": round(valu_tflops / VALU_PEAK_TFLOPS, 4),
                "valu_issue_frac_pmc": pmc_valu_issue(params),
                "valu_issue_source": SQ_PROFILE,
            },
        }
        if not args.no_parity:
            line["parity"] = parity_window(geom, params, cam_pos, image)
        if args.cpu_seconds > 0 and world == 1:  # the CPU baseline is an N=1 figure
            line["cpu_baseline"] = cpu_baseline(geom, params, cam_pos, args.cpu_seconds)
        print(json.dumps(line), flush=True)

    scene.close()
    ctx.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def parity_window(geom, params, cam_pos, image):
    """MAPE and bit-exactness of the GPU frame vs the CPU restatement on 4 windows."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle

    op = oracle.params_from(params)
    ocam = oracle.camera(cam_pos)
    wins = [(96, 64, 16, 16), (248, 248, 16, 16), (400, 300, 16, 16), (40, 440, 16, 16)]
    worst, exact = 0.0, True
    for (x, y, w, h) in wins:
        if x + w > params.width or y + h > params.height:
            continue
        ref, _ = oracle.render(geom, ocam, op, (x, y, w, h))
        got = image[y:y + h, x:x + w]
        worst = max(worst, rtmi.metrics.mape_f(ref, got))
        exact = exact and bool(np.array_equal(ref.view(np.uint32), got.view(np.uint32)))
    return {"mape_vs_cpu": worst, "bit_exact": exact, "windows": len(wins), "window_px": 16}


if __name__ == "__main__":
    main()
