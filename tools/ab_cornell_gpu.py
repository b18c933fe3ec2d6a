#!/usr/bin/env python3
"""Cornell box, GPU-engine preset (80 bounces), 512^2 x 256 spp: device-buffer frame time
of the librtmi.so named by RTMI_LIB (A/B of launcher choices), with the cast count and a
bit checksum of the image.

    RTMI_LIB=build/variants/x/librtmi.so python tools/ab_cornell_gpu.py [--split 16]
"""
import argparse
import hashlib
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "reinforcement-light-rays-pathtracer_amd"))
import rtmi  # noqa: E402

TILE = 32


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--split", type=int, default=16)
    ap.add_argument("--spp", type=int, default=256)
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    stream = torch.cuda.current_stream()
    g = rtmi.cornell_geometry(rtmi.RT_PRESET_GPU)
    p = rtmi.default_params(rtmi.RT_PRESET_GPU, width=512, height=512, spp=args.spp, spp_split=args.split)
    cam = rtmi.camera(rtmi.CAMERAS["cornell"])
    with rtmi.Context(0) as ctx, rtmi.Scene(ctx, g) as sc:
        tiles = rtmi.tiles.tile_origins(512, 512, TILE)
        out = torch.zeros((len(tiles), TILE, TILE, 3), dtype=torch.float32, device="cuda")
        casts = torch.zeros(1, dtype=torch.int64, device="cuda")
        fn = lambda: rtmi.render_tiles_device(ctx, sc, cam, p, tiles, TILE, out.data_ptr(), casts.data_ptr(),
                                              stream.cuda_stream)
        fn()
        torch.cuda.synchronize()
        ms = []
        for _ in range(args.rounds):
            casts.zero_()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            fn()
            e1.record(stream)
            torch.cuda.synchronize()
            ms.append(e0.elapsed_time(e1))
        c = int(casts.item())
        img = out.cpu().numpy()
    print(json.dumps({"lib": os.environ.get("RTMI_LIB", "default"), "ms": round(float(np.median(ms)), 3),
                      "ray_casts": c, "gcasts_s": round(c / float(np.median(ms)) / 1e6, 3),
                      "image_sha": hashlib.sha256(img.tobytes()).hexdigest()[:16]}), flush=True)


if __name__ == "__main__":
    main()
