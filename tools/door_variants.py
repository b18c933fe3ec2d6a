#!/usr/bin/env python3
"""Which door_room scene variant rendered the reference's Images/door_room/reference.png?

The reference comments scene blocks in and out by hand (GPU_Rendering_Engine/Source/
objects/object_importer.cu): the red material on triangles 24-35 (:152-155, commented at
HEAD), the blue on 12-23 (:161-163, active), the door-room lights (:214-237, commented) vs
the archway lights (:240-271, active at HEAD).  Each of the 8 combinations (rtmi.h
RT_DOOR_* bits) is rendered with the GPU-engine preset at the reference's 720x720 and
compared by 45x45-pixel block means of the 8-bit PutPixelSDL image with the reference's
renders (tests/golden/scenes_ref_stats.json): reference.png (the 4096-spp image the
thesis's MAPE values use) and default_128spp_50avg.png (its 128-spp default render).
--bounces sweeps MAX_RAY_BOUNCES for the default variant.

    python tools/door_variants.py [--spp 512] [--variants 0 1 ..] [--bounces 4 6 ..] [--save]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "reinforcement-light-rays-pathtracer_amd"))
import rtmi  # noqa: E402

WHITE_DOOR, NO_BLUE, ARCH = 1, 2, 4


def block_means(img):
    rgb8 = rtmi.metrics.argb_to_rgb8(rtmi.pack_argb(img)).astype(np.float64)
    return rgb8.reshape(16, 45, 16, 45, 3).mean(axis=(1, 3))


def compare(ours, ref):
    d = np.abs(ours - ref)
    scale = float((ours * ref).sum() / (ours * ours).sum())
    return {"block_mean_abs_diff": round(float(d.mean()), 3), "block_max_abs_diff": round(float(d.max()), 3),
            "fit_scale": round(scale, 4),
            "block_mean_abs_diff_after_scale": round(float(np.abs(ours * scale - ref).mean()), 3)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--spp", type=int, default=512)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "door_variants.json"))
    ap.add_argument("--save", action="store_true", help="also write each variant's image as PNG")
    ap.add_argument("--variants", type=int, nargs="*", default=list(range(8)))
    ap.add_argument("--bounces", type=int, nargs="*", default=[],
                    help="MAX_RAY_BOUNCES values to sweep for variant 0")
    args = ap.parse_args()
    stats = json.load(open(os.path.join(ROOT, "tests", "golden", "scenes_ref_stats.json")))
    refs = {k: np.array(stats[k]["means"]) for k in ("door_room", "door_room_default_128spp", "door_room_sarsa_128spp")
            if k in stats}
    cam = rtmi.camera(rtmi.CAMERAS["door_room"])
    res = {"spp": args.spp, "references": {k: {"file": stats[k]["file"], "mean": round(float(r.mean()), 3),
                                                "channel_means": [round(float(x), 3) for x in r.mean(axis=(0, 1))]}
                                            for k, r in refs.items()},
           "variants": [], "bounce_sweep": []}
    obj = os.path.join(ROOT, "assets", "models", "door_room.obj")
    runs = [(v, None) for v in args.variants] + [(0, b) for b in args.bounces]
    with rtmi.Context(0) as ctx:
        for v, bounces in runs:
            kw = {} if bounces is None else {"max_bounces": bounces}
            p = rtmi.default_params(rtmi.RT_PRESET_GPU, width=720, height=720, spp=args.spp, spp_split=16, **kw)
            g = rtmi.obj_geometry(obj, 1 | (v << 8))
            with rtmi.Scene(ctx, g) as sc:
                img, casts = rtmi.render(ctx, sc, cam, p)
            ours = block_means(img)
            e = {"variant": v, "max_bounces": p.max_bounces, "red_door": not (v & WHITE_DOOR),
                 "blue_block": not (v & NO_BLUE),
                 "lights": "archway (active at HEAD)" if v & ARCH else "door room (commented at HEAD)",
                 "mean": round(float(ours.mean()), 3),
                 "channel_means": [round(float(x), 3) for x in ours.mean(axis=(0, 1))],
                 "casts_per_sample": round(casts / (720 * 720 * args.spp), 3),
                 "vs": {k: compare(ours, r) for k, r in refs.items()}}
            e["block_means"] = np.round(ours, 2).tolist()
            if args.save:
                rtmi.save_png(os.path.join(os.path.dirname(args.out), f"door_variant{v}_b{p.max_bounces}.png"),
                              rtmi.pack_argb(img))
            (res["variants"] if bounces is None else res["bounce_sweep"]).append(e)
            print(json.dumps({k: x for k, x in e.items() if k != "block_means"}), flush=True)
    for k in refs:
        cands = res["variants"] + res["bounce_sweep"]
        best = min(cands, key=lambda e: e["vs"][k]["block_mean_abs_diff"])
        res["best_vs_" + k] = {"variant": best["variant"], "max_bounces": best["max_bounces"],
                                **best["vs"][k]}
        print("best vs", k, json.dumps(res["best_vs_" + k]))
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    json.dump(res, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
