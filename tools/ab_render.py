#!/usr/bin/env python3
"""In-process A/B timing of librtmi.so variants (guide §5.4 rule 24: interleaved
rounds in one process).  Each variant renders the Cornell 512^2/256-spp frame;
images must be bit-identical to the first variant's.

    python tools/ab_render.py build/variants/v0 build/variants/v1 ... [--rounds 5]
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "reinforcement-light-rays-pathtracer_amd"))
import rtmi  # noqa: E402
from rtmi import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--spp", type=int, default=256)
    ap.add_argument("--split", type=int, default=8)
    ap.add_argument("--scene", default="cornell")
    ap.add_argument("--preset", type=int, default=0)
    args = ap.parse_args()
    pkg = os.path.join(ROOT, "reinforcement-light-rays-pathtracer_amd")
    libs = []
    for v in args.variants:
        path = os.path.join(pkg, v, "librtmi.so") if not v.endswith(".so") else v
        L = ctypes.CDLL(path)
        _lib._declare(L)
        libs.append((v, L))
    if args.scene == "cornell":
        geom = rtmi.cornell_geometry(args.preset)
        cam_key = "cornell"
    else:
        geom = rtmi.obj_geometry(os.path.join(ROOT, "assets", "models", args.scene + ".obj"), args.scene)
        cam_key = args.scene
    p = rtmi.default_params(args.preset, width=512, height=512, spp=args.spp, spp_split=args.split)
    cam = rtmi.camera(rtmi.CAMERAS[cam_key])
    tiles = rtmi.tiles.rank_tiles(512, 512, 32, 0, 1)
    stream = torch.cuda.current_stream()
    fp = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))
    ip = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))
    state = []
    for name, L in libs:
        ctx, sc = ctypes.c_void_p(), ctypes.c_void_p()
        _lib.check(L.rt_ctx_create(0, ctypes.byref(ctx)))
        tri, alb = np.ascontiguousarray(geom.tri), np.ascontiguousarray(geom.albedo)
        lv, em = np.ascontiguousarray(geom.light), np.ascontiguousarray(geom.emission)
        grp = np.ascontiguousarray(geom.light_group)
        assert L.rt_scene_create(ctx, fp(tri), fp(alb), geom.n_surf, fp(lv), fp(em), ip(grp),
                                 geom.n_light, ctypes.byref(sc)) == 0
        out = torch.zeros((len(tiles), 32, 32, 3), device="cuda")
        casts = torch.zeros(1, dtype=torch.int64, device="cuda")
        state.append((name, L, ctx, sc, out, casts))

    def run(st):
        name, L, ctx, sc, out, casts = st
        t = np.ascontiguousarray(tiles)
        rc = L.rt_render_tiles_device(ctx, sc, ctypes.byref(cam), ctypes.byref(p), ip(t), len(t), 32,
                                      ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(casts.data_ptr()),
                                      ctypes.c_void_p(stream.cuda_stream))
        assert rc == 0, L.rt_last_error()

    for st in state:  # warm-up
        run(st)
    torch.cuda.synchronize()
    times = {st[0]: [] for st in state}
    for _ in range(args.rounds):
        for st in state:
            st[5].zero_()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            run(st)
            b.record(stream)
            torch.cuda.synchronize()
            times[st[0]].append(a.elapsed_time(b))
    ref = state[0][4].cpu().numpy()
    res = {}
    for st in state:
        img = st[4].cpu().numpy()
        c = int(st[5].item())
        ms = float(np.median(times[st[0]]))
        res[st[0]] = {"ms_median": round(ms, 4), "ms_min": round(min(times[st[0]]), 4),
                      "gcasts_s": round(c / ms / 1e6, 3), "same_image": bool(np.array_equal(img, ref))}
    print(json.dumps({"scene": args.scene, "preset": args.preset, "spp": args.spp, "results": res}))


if __name__ == "__main__":
    main()
