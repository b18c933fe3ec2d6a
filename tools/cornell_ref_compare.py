#!/usr/bin/env python3
"""Compare a GPU-preset Cornell render with the reference's own 720x720 renders
(tests/golden/cornell_ref_stats.json: 45x45-pixel block means of Images/cornell/*.png),
after the PutPixelSDL 8-bit packing.  Prints the block-mean differences per orientation."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "reinforcement-light-rays-pathtracer_amd"))
import rtmi  # noqa: E402


def blocks(img8, b=45):
    h, w, _ = img8.shape
    return img8[: h // b * b, : w // b * b].astype(np.float64).reshape(h // b, b, w // b, b, 3).mean(axis=(1, 3))


def main():
    spp = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    scene = sys.argv[2] if len(sys.argv) > 2 else "cornell"
    if scene == "cornell":
        ref = json.load(open(os.path.join(ROOT, "tests", "golden", "cornell_ref_stats.json")))
        geom = rtmi.cornell_geometry(rtmi.RT_PRESET_GPU)
        cam = rtmi.CAMERAS["cornell"]
    else:  # door_room, archway, complex_light_room
        key = "complex_light" if scene == "complex_light_room" else scene
        ref = {key: json.load(open(os.path.join(ROOT, "tests", "golden", "scenes_ref_stats.json")))[key]}
        geom = rtmi.obj_geometry(os.path.join(ROOT, "assets", "models", scene + ".obj"), scene)
        cam = rtmi.CAMERAS[scene]
    p = rtmi.default_params(rtmi.RT_PRESET_GPU, width=720, height=720, spp=spp, spp_split=16)
    with rtmi.Context(0) as ctx, rtmi.Scene(ctx, geom) as sc:
        img, casts = rtmi.render(ctx, sc, rtmi.camera(cam), p)
    rgb8 = rtmi.metrics.argb_to_rgb8(rtmi.pack_argb(img))
    ours = blocks(rgb8)
    for name, st in ref.items():
        r = np.array(st["means"])
        for tag, o in (("as is", ours), ("flip y", ours[::-1]), ("flip x", ours[:, ::-1]), ("transpose", ours.transpose(1, 0, 2))):
            d = np.abs(o - r)
            print(json.dumps({"scene": scene, "ref": name, "orient": tag, "spp": spp, "mean_abs": round(float(d.mean()), 3),
                              "max_abs": round(float(d.max()), 2), "ours_mean": round(float(o.mean()), 3),
                              "ref_mean": round(float(r.mean()), 3)}))


if __name__ == "__main__":
    main()
