#!/usr/bin/env python3
"""Probe: the Neural-Q renderer's first training rows (epsilon 1: uniform cells) at several
ENVIRONMENT_LIGHT values and cameras, for the statistics the reference logged at row 0
(door_room_12_12_stats.txt: 50.335 / 203,255 zero; cornell_stats_12_12.txt: 8.07179 / 218,999)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "reinforcement-light-rays-pathtracer_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import rtmi  # noqa: E402
from nq_pin import geometry  # noqa: E402

out = []
with rtmi.Context(0) as ctx:
    for scene in ("door_room", "cornell"):
        g = geometry(scene)
        for env in (0.0, 0.25, 1.0):
            W0, b0 = rtmi.dqn.glorot_weights(g.nn_vertices.size)
            with rtmi.Scene(ctx, g) as sc, rtmi.dqn.DqnTrainer(ctx, g.nn_vertices, W0, b0) as tr, \
                    rtmi.dqn.NeuralQ(ctx, sc, tr, epsilon_start=1.0, epsilon_min=0.05, epsilon_decay=0.01) as nq:
                p = rtmi.default_params(rtmi.RT_PRESET_GPU, width=720, height=720, spp=2)
                p.env_light = env
                _, st, casts = nq.render_frame(rtmi.camera(rtmi.CAMERAS[scene]), p)
                r = {"scene": scene, "env": env, "rows": st.tolist(), "casts_per_sample": casts / (720 * 720 * 2)}
                print(json.dumps(r), flush=True)
                out.append(r)
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
json.dump(out, open(os.path.join(ROOT, "gpurun_out", "nq_env_probe.json"), "w"), indent=1)
