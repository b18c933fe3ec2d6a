#!/usr/bin/env python3
"""Neural-Q training (BASELINE north star (f) item 1) against the reference's own training logs.

Radiance_Map_Data/{door_room_12_12_stats,cornell_stats_12_12,archway_12_12,complex_light_room_12_12}.txt
(tests/golden/nn_ref_stats.json) hold one row per training sample, written by
NeuralQPathtracer::render_frame (GPU/deep_learning/neural_q_pathtracer.cu:545-583): the average
path length (sum of ray_bounces / pixels), the loss summed over the sample's learning steps, and
the zero-contribution paths.  The rows fall linearly (door room 50.3 -> 33.5 over 100 rows) and
flatten at the end: epsilon-greedy from epsilon 1 decayed by EPSILON_DECAY 0.01 per sample down to
EPSILON_MIN 0.05 (deep_learning_settings.h:5-8; the thesis's ε = 1 start, 4_critical_evaluation.tex).
This runs rt_neuralq_render_frame at those settings -- 720 x 720, GPU-engine preset, batch 4096
(main.cu:116-124), DyNet's Adam defaults, the network from DyNet's default Glorot initialisation
(rtmi.dqn.glorot_weights) or He-normal -- one sample per row, and records each row next to the log.

    python tools/nq_pin.py [--scenes door_room cornell] [--rows 100] [--seeds 1984] [--init glorot]
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

LOGS = {"door_room": "door_room_12_12", "cornell": "cornell_12_12", "archway": "archway_12_12",
        "complex_light_room": "complex_light_room_12_12"}


def geometry(scene):
    if scene == "cornell":
        return rtmi.cornell_geometry(rtmi.RT_PRESET_GPU)
    return rtmi.obj_geometry(os.path.join(ROOT, "assets", "models", scene + ".obj"), scene)


def run(ctx, scene, rows, seed, init, size=720, batch=4096, eps=(1.0, 0.05, 0.01), lr=1e-3, log=print):
    """one training run: per row (sample) the average path length, loss and zero-contribution paths"""
    g = geometry(scene)
    cam = rtmi.camera(rtmi.CAMERAS[scene])
    n_in = g.nn_vertices.size
    W0, b0 = (rtmi.dqn.glorot_weights if init == "glorot" else rtmi.dqn.synthetic_weights)(n_in, seed=seed)
    out = {"path": [], "loss": [], "zero": [], "s": []}
    with rtmi.Scene(ctx, g) as sc, rtmi.dqn.DqnTrainer(ctx, g.nn_vertices, W0, b0, learning_rate=lr) as tr, \
            rtmi.dqn.NeuralQ(ctx, sc, tr, batch_size=batch, epsilon_start=eps[0], epsilon_min=eps[1],
                             epsilon_decay=eps[2]) as nq:
        p = rtmi.default_params(rtmi.RT_PRESET_GPU, width=size, height=size, spp=1, seed=seed)
        for r in range(rows):
            t0 = time.perf_counter()
            _, stats, _ = nq.render_frame(cam, p)
            out["path"].append(round(float(stats[0, 0]), 4))
            out["loss"].append(float(stats[0, 1]))
            out["zero"].append(int(stats[0, 2]))
            out["s"].append(round(time.perf_counter() - t0, 2))
            log(f"{scene} seed {seed} row {r}: {out['path'][-1]} {out['loss'][-1]:.4g} {out['zero'][-1]} ({out['s'][-1]} s)")
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scenes", nargs="*", default=["door_room", "cornell"])
    ap.add_argument("--rows", type=int, default=0, help="rows per run (0: the log's length)")
    ap.add_argument("--seeds", type=int, nargs="*", default=[1984])
    ap.add_argument("--init", default="glorot", choices=["glorot", "he"])
    ap.add_argument("--lr", type=float, default=1e-3, help="Adam's learning rate (DyNet's default 1e-3; 0: a network that never learns)")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "nq_pin.json"))
    args = ap.parse_args()
    ref = json.load(open(os.path.join(ROOT, "tests", "golden", "nn_ref_stats.json")))
    res = {"settings": {"size": 720, "batch": 4096, "epsilon": [1.0, 0.05, 0.01], "init": args.init, "lr": args.lr,
                        "preset": "gpu"}, "runs": []}
    os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
    with rtmi.Context(0) as ctx:
        for scene in args.scenes:
            log = ref[LOGS[scene]]
            rows = args.rows or len(log["avg_path_length"])
            for seed in args.seeds:
                r = run(ctx, scene, rows, seed, args.init, lr=args.lr, log=lambda m: print(m, flush=True))
                r.update({"scene": scene, "seed": seed, "ref_path": log["avg_path_length"][:rows],
                          "ref_zero": log["zero_contribution_paths"][:rows]})
                res["runs"].append(r)
                json.dump(res, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
