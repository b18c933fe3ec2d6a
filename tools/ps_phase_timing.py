#!/usr/bin/env python3
"""Where k_render_ps's time goes: the bench frame (Cornell 512^2, 256 spp, CPU preset,
split 64) at MAX_RAY_BOUNCES 0, 1 and 2 (primaries only, + one bounce, the bench), HIP
events around the tile render, median of 5."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "reinforcement-light-rays-pathtracer_amd"))
import rtmi  # noqa: E402


def main():
    g = rtmi.cornell_geometry(rtmi.RT_PRESET_CPU)
    cam = rtmi.camera(rtmi.CAMERAS["cornell"])
    stream = torch.cuda.current_stream()
    out = torch.zeros((256, 32, 32, 3), device="cuda")
    casts = torch.zeros(1, dtype=torch.int64, device="cuda")
    tiles = rtmi.tiles.tile_origins(512, 512, 32)
    res = {}
    with rtmi.Context(0) as ctx, rtmi.Scene(ctx, g) as sc:
        for mb in (0, 1, 2):
            p = rtmi.default_params(rtmi.RT_PRESET_CPU, width=512, height=512, spp=256, spp_split=64, max_bounces=mb)
            ts = []
            for it in range(6):
                casts.zero_()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                rtmi.render_tiles_device(ctx, sc, cam, p, tiles, 32, out.data_ptr(), casts.data_ptr(), stream.cuda_stream)
                e1.record(stream)
                torch.cuda.synchronize()
                if it:
                    ts.append(e0.elapsed_time(e1))
            ms = float(np.median(ts))
            c = int(casts.item())
            res[mb] = {"ms": round(ms, 3), "casts": c, "gcasts_s": round(c / ms / 1e6, 2)}
            print(mb, json.dumps(res[mb]), flush=True)
    d1 = res[1]["ms"] - res[0]["ms"]
    d2 = res[2]["ms"] - res[1]["ms"]
    print(json.dumps({"primary_ms": res[0]["ms"], "bounce1_ms": round(d1, 3), "bounce2_ms": round(d2, 3),
                      "ns_per_primary": round(res[0]["ms"] * 1e6 / res[0]["casts"], 4),
                      "ns_per_bounce1_cast": round(d1 * 1e6 / max(1, res[1]["casts"] - res[0]["casts"]), 4),
                      "ns_per_bounce2_cast": round(d2 * 1e6 / max(1, res[2]["casts"] - res[1]["casts"]), 4)}))


if __name__ == "__main__":
    main()
