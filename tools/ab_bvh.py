#!/usr/bin/env python3
"""In-process A/B timing of librtmi.so variants on the BVH workload (bunny in the Cornell
box, GPU preset, 256^2 x 16 spp; CPU preset 256^2 x 16 spp), plus the filter scan.

    python tools/ab_bvh.py build/variants/v0 build/variants/v1 ... [--rounds 3]
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "reinforcement-light-rays-pathtracer_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import rtmi  # noqa: E402
from rtmi import _lib  # noqa: E402
from test_bvh import bunny_cornell  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--spp", type=int, default=16)
    args = ap.parse_args()
    pkg = os.path.join(ROOT, "reinforcement-light-rays-pathtracer_amd")
    fp = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))
    ip = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))
    res = {}
    for preset in (1, 0):
        g = bunny_cornell(rtmi, preset)
        p = rtmi.default_params(preset, width=args.size, height=args.size, spp=args.spp, spp_split=8)
        cam = rtmi.camera(rtmi.CAMERAS["cornell"])
        tiles = np.ascontiguousarray(rtmi.tiles.rank_tiles(args.size, args.size, 32, 0, 1), np.int32)
        out = torch.zeros((len(tiles), 32, 32, 3), device="cuda")
        casts = torch.zeros(1, dtype=torch.int64, device="cuda")
        for v in args.variants:
            path = os.path.join(pkg, v, "librtmi.so")
            L = ctypes.CDLL(path)
            _lib._declare(L)
            ctx, sc = ctypes.c_void_p(), ctypes.c_void_p()
            assert L.rt_ctx_create(0, ctypes.byref(ctx)) == 0
            tri, alb = np.ascontiguousarray(g.tri), np.ascontiguousarray(g.albedo)
            lv, em, grp = np.ascontiguousarray(g.light), np.ascontiguousarray(g.emission), np.ascontiguousarray(g.light_group)
            assert L.rt_scene_create(ctx, fp(tri), fp(alb), g.n_surf, fp(lv), fp(em), ip(grp), g.n_light,
                                     ctypes.byref(sc)) == 0
            for mode, name in ((2, "bvh"), (1, "scan")):
                if name == "scan" and v != args.variants[0]:
                    continue
                assert L.rt_scene_set_accel(sc, mode) == 0
                ts = []
                for r in range(args.rounds + 1):
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    rc = L.rt_render_tiles_device(ctx, sc, ctypes.byref(cam), ctypes.byref(p), ip(tiles), len(tiles), 32,
                                                  ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(casts.data_ptr()),
                                                  ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
                    assert rc == 0
                    torch.cuda.synchronize()
                    if r:
                        ts.append(time.perf_counter() - t0)
                res[f"p{preset}:{v}:{name}"] = round(min(ts) * 1e3, 2)
            L.rt_scene_destroy(sc)
            L.rt_ctx_destroy(ctx)
        print(json.dumps(res), flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
