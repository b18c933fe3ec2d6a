#!/usr/bin/env python3
"""Expected-SARSA learning trajectory against the reference's own training logs.

Radiance_Map_Data/sarsa_{cornell,door_scene,archway,complex_light_scene}.txt hold one line per
training frame (GPU/main.cu:321-339): the average path length (integer division of the sum of
per-pixel int(mean path length) by the pixel count), 0.0, and the zero-contribution paths
(samples whose mean radiance is below THROUGHPUT_THRESHOLD, reinforcement_path_tracing.cu:36-42);
tests/golden/sarsa_ref_stats.json keeps them.  The logs do not state the spp of those runs;
the zero-contribution count is a count of samples, so its ratio to ours at a known spp gives it.

For each scene, TD rule (frame-synchronous, in-frame) and spp this renders frames 0..F-1 at the
reference's 720x720 with the GPU-engine preset and records each frame's logged statistic and
zero count next to the reference's, plus the block means of the last frame.

    python tools/sarsa_pin.py [--frames 8] [--spp 1 32] [--seeds 1984] [--areas 0.001 0.1] [--out gpurun_out/sarsa_pin]
"""
import argparse
import itertools
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "reinforcement-light-rays-pathtracer_amd"))
import rtmi  # noqa: E402

MODELS = os.path.join(ROOT, "assets", "models")
SCENES = ("cornell", "door_room", "archway", "complex_light_room")


def geometry(spec):
    """scene[:variant]: variant = the rt_obj_geometry RT_DOOR_* bits of door_room"""
    scene, _, var = spec.partition(":")
    if scene == "cornell":
        return rtmi.cornell_geometry(rtmi.RT_PRESET_GPU)
    kind = rtmi.OBJ_KINDS[scene] | (int(var or 0) << 8)
    return rtmi.obj_geometry(os.path.join(MODELS, scene + ".obj"), kind)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=8)
    ap.add_argument("--spp", type=int, nargs="*", default=[1, 32])
    ap.add_argument("--seeds", type=int, nargs="*", default=[1984])
    ap.add_argument("--modes", nargs="*", default=["frame", "inframe"])
    ap.add_argument("--scenes", nargs="*", default=list(SCENES))
    ap.add_argument("--size", type=int, default=720)
    ap.add_argument("--lanes", type=int, nargs="*", default=[0],
                    help="in-frame rule: paths in flight (rt_sarsa_set_inframe_lanes; 0 = the whole device)")
    ap.add_argument("--areas", type=float, nargs="*", default=[0.001],
                    help="AREA_PER_SAMPLE values (radiance_volumes_settings.h:12) to sweep")
    ap.add_argument("--final-spp", type=int, default=0,
                    help="after the frames, one frame at this spp compared with the reference's SARSA render")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "sarsa_pin"))
    args = ap.parse_args()
    os.makedirs(args.out, exist_ok=True)
    ref = json.load(open(os.path.join(ROOT, "tests", "golden", "sarsa_ref_stats.json")))
    imgs = json.load(open(os.path.join(ROOT, "tests", "golden", "scenes_ref_stats.json")))
    png_key = {"cornell": "cornell_sarsa_128spp", "door_room": "door_room_sarsa_128spp",
               "archway": "archway_sarsa_128spp", "complex_light_room": "complex_light_sarsa_128spp"}
    W = H = args.size
    res = {"size": W, "frames": args.frames, "runs": []}
    with rtmi.Context(0) as ctx:
        for spec in args.scenes:
            g = geometry(spec)
            scene = spec.partition(":")[0]
            cam = rtmi.camera(rtmi.CAMERAS[scene])
            with rtmi.Scene(ctx, g) as sc:
                for area, mode, spp, seed, lanes in itertools.product(args.areas, args.modes, args.spp, args.seeds,
                                                                      args.lanes):
                    if mode != "inframe" and lanes != args.lanes[0]:
                        continue
                    rm = rtmi.sarsa.RadianceMap(ctx, sc, 1984, area_per_sample=area)  # placement seed fixed
                    try:
                        if mode == "inframe":
                            rm.set_td_mode(rtmi.sarsa.TD_INFRAME)
                            rm.set_inframe_lanes(lanes)
                        p = rtmi.default_params(rtmi.RT_PRESET_GPU, width=W, height=H, spp=spp,
                                                spp_split=min(spp, 8), seed=seed)
                        logged, zero, cps, ms = [], [], [], []
                        for f in range(args.frames):
                            t = time.time()
                            img, casts = rm.render(cam, p, 1)
                            ms.append(round((time.time() - t) * 1e3, 1))
                            paths, z = rm.frame_stats()
                            logged.append(paths // (W * H))
                            zero.append(z)
                            cps.append(round(casts / (W * H * spp), 4))
                        final = None
                        if args.final_spp:
                            pf = rtmi.default_params(rtmi.RT_PRESET_GPU, width=W, height=H,
                                                     spp=args.final_spp, spp_split=8, seed=seed)
                            img, casts = rm.render(cam, pf, 1)
                            paths, z = rm.frame_stats()
                            rgb8 = rtmi.metrics.argb_to_rgb8(rtmi.pack_argb(img)).astype(np.float64)
                            final = {"spp": args.final_spp, "logged_avg_path": paths // (W * H),
                                     "casts_per_sample": round(casts / (W * H * args.final_spp), 4),
                                     "mean8": round(float(rgb8.mean()), 3)}
                            key = png_key[scene]
                            if W == 720 and key in imgs:
                                bm = rgb8.reshape(16, 45, 16, 45, 3).mean(axis=(1, 3))
                                rb = np.array(imgs[key]["means"])
                                d = np.abs(bm - rb)
                                final.update({"ref_png": imgs[key]["file"], "ref_mean8": round(float(rb.mean()), 3),
                                              "block_mean_abs_diff": round(float(d.mean()), 3),
                                              "block_max_abs_diff": round(float(d.max()), 3)})
                        r = {"scene": spec, "final": final, "mode": mode, "spp": spp, "seed": seed,
                             "area_per_sample": area, "n_volumes": rm.n_volumes,
                             "inframe_lanes": lanes if mode == "inframe" else None,
                             "logged_avg_path": logged, "zero_paths": zero,
                             "zero_frac": [round(z / (W * H * spp), 5) for z in zero],
                             "casts_per_sample": cps, "ms": ms,
                             "ref_avg_path": ref[scene]["avg_path_length"][:args.frames],
                             "ref_zero_paths": ref[scene]["zero_contribution_paths"][:args.frames],
                             "mean8": float(rtmi.metrics.argb_to_rgb8(rtmi.pack_argb(img)).mean())}
                        res["runs"].append(r)
                        print(json.dumps(r), flush=True)
                    finally:
                        rm.close()
    with open(os.path.join(args.out, "sarsa_pin.json"), "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
