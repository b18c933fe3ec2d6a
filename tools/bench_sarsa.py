#!/usr/bin/env python3
"""Expected-SARSA path measurements (BASELINE config 3: door_room 512^2, 256 spp).

    python tools/bench_sarsa.py [--scene door_room] [--width 512] [--spp 256] [--frames 4]

One frame = draw_reinforcement_path_tracing over the image (spp samples per pixel)
+ the Q-table/CDF update.  Prints one JSON line: per-frame ms, Mrays/s, average path
length per frame (the reference logs the same statistic, Radiance_Map_Data/sarsa_*.txt).
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "reinforcement-light-rays-pathtracer_amd"))
import rtmi  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="door_room")
    ap.add_argument("--width", type=int, default=512)
    ap.add_argument("--spp", type=int, default=256)
    ap.add_argument("--split", type=int, default=8)
    ap.add_argument("--frames", type=int, default=4)
    ap.add_argument("--tile", type=int, default=32)
    ap.add_argument("--search", choices=("grid", "kd"), default="grid")
    ap.add_argument("--lib", default=None, help="librtmi.so variant directory (A/B timing)")
    args = ap.parse_args()
    if args.lib:
        rtmi._lib.LIB_PATH = os.path.join(ROOT, "reinforcement-light-rays-pathtracer_amd", args.lib, "librtmi.so")
    if args.scene == "cornell":
        g = rtmi.cornell_geometry(rtmi.RT_PRESET_GPU)
    else:
        g = rtmi.obj_geometry(os.path.join(ROOT, "assets", "models", args.scene + ".obj"), args.scene)
    ctx = rtmi.Context(0)
    sc = rtmi.Scene(ctx, g)
    rm = rtmi.sarsa.RadianceMap(ctx, sc, 1984)
    rm.set_search(rtmi.sarsa.SEARCH_GRID if args.search == "grid" else rtmi.sarsa.SEARCH_KD)
    p = rtmi.default_params(rtmi.RT_PRESET_GPU, width=args.width, height=args.width, spp=args.spp,
                            spp_split=args.split)
    cam = rtmi.camera(rtmi.CAMERAS[args.scene])
    T = args.tile
    tiles = rtmi.tiles.tile_origins(args.width, args.width, T)
    stream = torch.cuda.current_stream()
    out = torch.zeros((len(tiles), T, T, 3), dtype=torch.float32, device="cuda")
    casts = torch.zeros(1, dtype=torch.int64, device="cuda")
    frames = []
    for f in range(args.frames):
        casts.zero_()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        rm.render_tiles_device(cam, p, tiles, T, out.data_ptr(), casts.data_ptr(), True, stream.cuda_stream)
        e1.record(stream)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1)
        c = int(casts.item())
        frames.append({"frame": f, "ms": round(ms, 3), "mrays_s": round(c / (ms * 1e-3) / 1e6, 1),
                       "avg_path_length": round(c / (args.width * args.width * args.spp), 3),
                       "image_mean": round(float(out.mean().item()), 5)})
        print(json.dumps(frames[-1]), file=sys.stderr, flush=True)
    q, cdf, vis, acc = rm.read()
    res = {"lib": args.lib or "build", "scene": args.scene, "width": args.width, "spp": args.spp, "volumes": rm.n_volumes,
           "frames": frames, "search": rm.search_stats(), "visits": int(vis.sum()), "q_max": float(q.max()),
           "finite": bool(np.isfinite(out.cpu().numpy()).all())}
    print(json.dumps(res))
    rm.close()
    sc.close()
    ctx.close()


if __name__ == "__main__":
    main()
