#!/usr/bin/env python3
"""Pin the DQN renderer (rt_render_dqn) against the reference's own NN renders.

The reference ships three trained networks (Radiance_Map_Data/*.model, DyNet text format)
and the renders its pretrained renderer made with two of them:
  door_room_12_12.model -> Images/door_room/nn_128spp_32avg.png  ("32avg": the render's
                           average path length, pre_trained_pathtracer.cu:366-375)
  cornell_12_12.model   -> Images/cornell/nn_128spp_avg.png
and the default renders of the same scenes (default_128spp_50avg.png, default_128spp_6avg.png).

For each scene this renders, at the reference's 720x720 and GPU-engine preset:
  default   uniform sampling (rt_render), the same spp
  trained   the shipped network through rt_render_dqn
  transposed  the same parameters read in the other matrix order (row- instead of
            column-major: the DyNet order error this gate must see)
  synthetic He-normal weights (an untrained network)
  gt        uniform sampling at --gt-spp (converged ground truth)
and reports casts per sample, the 45x45 block means against the reference's PNGs, and the
noise of each render (MAPE of the 8-bit image against the ground truth, the metric of
Graphing/mape.py), next to the same noise figure of the reference's own PNGs.

    python tools/nn_pin.py [--spp 128] [--gt-spp 4096] [--out gpurun_out/nn_pin]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "reinforcement-light-rays-pathtracer_amd"))
import rtmi  # noqa: E402

MODELS = os.path.join(ROOT, "assets", "models")


def rgb8(img):
    return rtmi.metrics.argb_to_rgb8(rtmi.pack_argb(img))


def block_means(a8):
    return a8.astype(np.float64).reshape(16, 45, 16, 45, 3).mean(axis=(1, 3))


def transposed(W):
    """each weight matrix read in the wrong order: its column-major bytes taken row-major"""
    return [np.ascontiguousarray(w.ravel(order="F").reshape(w.shape)) for w in W]


def scene(name):
    if name == "cornell":
        g = rtmi.cornell_geometry(rtmi.RT_PRESET_GPU)
        return g, rtmi.camera(rtmi.CAMERAS["cornell"])
    return rtmi.obj_geometry(os.path.join(MODELS, f"{name}.obj"), name), rtmi.camera(rtmi.CAMERAS[name])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--spp", type=int, default=128)
    ap.add_argument("--gt-spp", type=int, default=4096)
    ap.add_argument("--scenes", nargs="*", default=["door_room", "cornell"])
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "nn_pin"))
    args = ap.parse_args()
    os.makedirs(args.out, exist_ok=True)
    models = {"door_room": ["door_room_12_12.model"], "cornell": ["cornell_12_12.model", "cornell_no_decay.model"]}
    res = {"spp": args.spp, "gt_spp": args.gt_spp}
    with rtmi.Context(0) as ctx:
        for name in args.scenes:
            g, cam = scene(name)
            p = rtmi.default_params(rtmi.RT_PRESET_GPU, width=720, height=720, spp=args.spp, spp_split=16)
            pg = rtmi.default_params(rtmi.RT_PRESET_GPU, width=720, height=720, spp=args.gt_spp, spp_split=16)
            out = {}
            imgs = {}
            with rtmi.Scene(ctx, g) as sc:
                t = time.time()
                gt, gc = rtmi.render(ctx, sc, cam, pg)
                out["gt"] = {"casts_per_sample": gc / (720 * 720 * args.gt_spp), "s": time.time() - t}
                imgs["gt"] = gt
                d, dc = rtmi.render(ctx, sc, cam, p)
                out["default"] = {"casts_per_sample": dc / (720 * 720 * args.spp)}
                imgs["default"] = d
                nnv = g.nn_vertices
                runs = []
                for m in models[name]:
                    W, b = rtmi.dqn.split_layers(rtmi.dqn.read_dynet(os.path.join(MODELS, m)))
                    runs.append((m, W, b))
                    runs.append((m + ":transposed", transposed(W), b))
                runs.append(("synthetic", *rtmi.dqn.synthetic_weights(nnv.size)))
                for key, W, b in runs:
                    t = time.time()
                    with rtmi.dqn.Dqn(ctx, nnv, W, b) as net:
                        img, casts = rtmi.dqn.render(ctx, sc, net, cam, p)
                    out[key] = {"casts_per_sample": casts / (720 * 720 * args.spp), "s": time.time() - t}
                    imgs[key] = img
            g8 = rgb8(imgs["gt"])
            stats = json.load(open(os.path.join(ROOT, "tests", "golden", "scenes_ref_stats.json")))
            refs = {"nn_png": stats[f"{name}_nn_128spp"], "default_png": stats[f"{name}_default_128spp"]}
            for key, img in imgs.items():
                a8 = rgb8(img)
                out[key]["mape_vs_gt"] = rtmi.metrics.mape8(g8, a8)
                out[key]["mean8"] = float(a8.mean())
                for rk, rv in refs.items():
                    d = np.abs(block_means(a8) - np.array(rv["means"]))
                    out[key][f"vs_{rk}"] = {"file": rv["file"], "block_mean_abs_diff": round(float(d.mean()), 3),
                                            "block_max_abs_diff": round(float(d.max()), 3)}
                np.save(os.path.join(args.out, f"{name}_{key.replace(':', '_')}.npy"), a8)
            res[name] = out
            print(name, json.dumps(out, indent=1), flush=True)
    with open(os.path.join(args.out, "nn_pin.json"), "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
