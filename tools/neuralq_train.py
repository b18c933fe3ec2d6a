#!/usr/bin/env python3
"""Train a Q-network with the Neural-Q renderer on a scene, then render with it.

    python tools/neuralq_train.py [--scene door_room] [--size 720] [--frames 3] [--spp 4]
                                  [--eval-spp 16] [--out gpurun_out/neuralq_train.json]

1. NeuralQPathtracer frames (rt_neuralq_render_frame) starting from synthetic He-normal
   weights (the reference starts DQNetwork from DyNet's initialisation): per-sample stats
   rows (nn_training_stats.txt) go to the JSON and to <out>.stats.txt.
2. The pretrained-network renderer (rt_render_dqn, config 4's sampler) at --eval-spp with
   (a) the synthetic weights, (b) the trained weights, (c) uniform sampling (the GPU
   preset): MAPE of each against a converged reference -- the door room's own 128-spp
   render block means (Images/door_room/default_128spp_50avg.png, 45x45 blocks) at 720,
   and our 1024-spp uniform render at the same size -- at equal spp.  Lower is better.
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


def mape(a, ref):
    return float(np.mean(np.abs(a - ref) / np.maximum(ref, 1e-3)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="door_room")
    ap.add_argument("--size", type=int, default=720)
    ap.add_argument("--frames", type=int, default=3)
    ap.add_argument("--spp", type=int, default=4)
    ap.add_argument("--eval-spp", type=int, default=16)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--lr", type=float, default=1e-3)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "neuralq_train.json"))
    args = ap.parse_args()
    g = rtmi.obj_geometry(os.path.join(ROOT, "assets", "models", args.scene + ".obj"), args.scene)
    cam = rtmi.camera(rtmi.CAMERAS[args.scene])
    W0, b0 = rtmi.dqn.synthetic_weights(g.nn_vertices.size)
    res = {"scene": args.scene, "size": args.size, "frames": args.frames, "spp_per_frame": args.spp,
           "batch": args.batch, "lr": args.lr, "eval_spp": args.eval_spp, "train": []}
    S = args.size
    with rtmi.Context(0) as ctx, rtmi.Scene(ctx, g) as sc:
        with rtmi.dqn.DqnTrainer(ctx, g.nn_vertices, W0, b0, learning_rate=args.lr) as tr:
            with rtmi.dqn.NeuralQ(ctx, sc, tr, batch_size=args.batch) as nq:
                p = rtmi.default_params(rtmi.RT_PRESET_GPU, width=S, height=S, spp=args.spp)
                lines = []
                for f in range(args.frames):
                    t0 = time.perf_counter()
                    img, stats, casts = nq.render_frame(cam, p)
                    dt = time.perf_counter() - t0
                    lines.append(rtmi.dqn.NeuralQ.stats_lines(stats))
                    row = {"frame": f, "s": round(dt, 2), "ray_casts": casts,
                           "avg_path_length": [round(float(x), 3) for x in stats[:, 0]],
                           "loss": [float(x) for x in stats[:, 1]],
                           "zero_contribution": [int(x) for x in stats[:, 2]], "epsilon": nq.epsilon}
                    res["train"].append(row)
                    print(json.dumps(row), flush=True)
            W1, b1 = tr.params()
        with open(args.out + ".stats.txt", "w") as fh:
            fh.write("".join(lines))
        pe = rtmi.default_params(rtmi.RT_PRESET_GPU, width=S, height=S, spp=args.eval_spp)
        pr = rtmi.default_params(rtmi.RT_PRESET_GPU, width=S, height=S, spp=1024, spp_split=16)
        ref, _ = rtmi.render(ctx, sc, cam, pr)
        evals = {}
        for name, (W, b) in (("synthetic", (W0, b0)), ("trained", (W1, b1))):
            with rtmi.dqn.Dqn(ctx, g.nn_vertices, W, b) as net:
                img, casts = rtmi.dqn.render(ctx, sc, net, cam, pe)
            evals[name] = (img, casts)
        uni, ucasts = rtmi.render(ctx, sc, cam, pe)
        evals["uniform"] = (uni, ucasts)
    key = {"door_room": "door_room_default_128spp", "archway": "archway", "complex_light_room": "complex_light"}
    stats_ref = json.load(open(os.path.join(ROOT, "tests", "golden", "scenes_ref_stats.json"))).get(key.get(args.scene))
    res["eval"] = {}
    for name, (img, casts) in evals.items():
        e = {"mape_vs_1024spp_uniform": round(mape(img, ref), 4), "ray_casts": casts,
             "casts_per_sample": round(casts / (S * S * args.eval_spp), 3), "mean": float(img.mean())}
        if stats_ref is not None and S == 720:
            rgb8 = rtmi.metrics.argb_to_rgb8(rtmi.pack_argb(img)).astype(np.float64)
            bm = rgb8.reshape(16, 45, 16, 45, 3).mean(axis=(1, 3))
            refb = np.array(stats_ref["means"])
            e["block_mean_abs_diff_vs_" + stats_ref["file"].split("/")[-1]] = round(float(np.abs(bm - refb).mean()), 3)
        res["eval"][name] = e
        print(name, json.dumps(e), flush=True)
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    json.dump(res, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
