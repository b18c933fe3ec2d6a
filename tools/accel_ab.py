#!/usr/bin/env python3
"""Frame time of one scene with the library's default closest-hit choice (ACCEL_AUTO: the
matrix-core / fp32 filter up to 256 triangles) against the exact BVH forced on
(ACCEL_BVH), same library, same frame; the images and ray casts must be identical.

    python tools/accel_ab.py --scene complex_light_room --preset 1 --size 512 --spp 256 --split 8
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
    ap.add_argument("--scene", default="complex_light_room")
    ap.add_argument("--preset", type=int, default=1)
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--spp", type=int, default=256)
    ap.add_argument("--split", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    if args.scene == "cornell":
        geom, key = rtmi.cornell_geometry(args.preset), "cornell"
    else:
        geom = rtmi.obj_geometry(os.path.join(ROOT, "assets", "models", args.scene + ".obj"), args.scene)
        key = args.scene
    W = args.size
    p = rtmi.default_params(args.preset, width=W, height=W, spp=args.spp, spp_split=args.split)
    cam = rtmi.camera(rtmi.CAMERAS[key])
    tiles = rtmi.tiles.rank_tiles(W, W, 32, 0, 1)
    stream = torch.cuda.current_stream()
    res = {}
    with rtmi.Context(0) as ctx, rtmi.Scene(ctx, geom) as sc:
        for name, mode in (("auto", rtmi.ACCEL_AUTO), ("bvh", rtmi.ACCEL_BVH)):
            sc.set_accel(mode)
            out = torch.zeros((len(tiles), 32, 32, 3), device="cuda")
            casts = torch.zeros(1, dtype=torch.int64, device="cuda")
            times = []
            for _ in range(args.rounds + 1):
                casts.zero_()
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(stream)
                rtmi.render_tiles_device(ctx, sc, cam, p, tiles, 32, out.data_ptr(), casts.data_ptr(),
                                         stream.cuda_stream)
                b.record(stream)
                torch.cuda.synchronize()
                times.append(a.elapsed_time(b))
            res[name] = {"ms_median": round(float(np.median(times[1:])), 3), "casts": int(casts.item()),
                         "img": out.cpu().numpy()}
    same = bool(np.array_equal(res["auto"]["img"].view(np.uint32), res["bvh"]["img"].view(np.uint32)))
    print(json.dumps({"scene": args.scene, "preset": args.preset, "size": W, "spp": args.spp,
                      "triangles": geom.n_tri, "auto_ms": res["auto"]["ms_median"], "bvh_ms": res["bvh"]["ms_median"],
                      "casts_equal": res["auto"]["casts"] == res["bvh"]["casts"], "same_image": same}))


if __name__ == "__main__":
    main()
