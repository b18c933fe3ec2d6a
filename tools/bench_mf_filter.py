#!/usr/bin/env python3
"""The bounce-cast hit test alone: fp32 two-phase filter (k_intersect) vs the matrix-core
filter (k_intersect_mf, rt_intersect_method) on bounce-like rays of a scene (origins on
surface triangles, directions into their hemisphere).  Run it under
`rocprofv3 --kernel-trace --stats` for the kernel times; prints the candidate counts.

    python tools/bench_mf_filter.py [--scene cornell] [--n 4194304] [--reps 3]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "reinforcement-light-rays-pathtracer_amd"))
import rtmi  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="cornell")
    ap.add_argument("--n", type=int, default=1 << 22)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    if args.scene == "cornell":
        g = rtmi.cornell_geometry(rtmi.RT_PRESET_CPU)
    else:
        g = rtmi.obj_geometry(os.path.join(ROOT, "assets", "models", args.scene + ".obj"), args.scene)
    n = args.n
    rng = np.random.default_rng(0)
    tri = g.tri.reshape(-1, 3, 3).astype(np.float64)
    k = rng.integers(0, tri.shape[0], n)
    a1, a2 = rng.random(n), rng.random(n)
    flip = a1 + a2 > 1
    a1[flip], a2[flip] = 1 - a1[flip], 1 - a2[flip]
    v = tri[k]
    pos = v[:, 0] + a1[:, None] * (v[:, 1] - v[:, 0]) + a2[:, None] * (v[:, 2] - v[:, 0])
    nrm = np.cross(v[:, 1] - v[:, 0], v[:, 2] - v[:, 0])
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    d *= np.sign(np.sum(d * nrm, axis=1, keepdims=True))
    o = (pos + 1e-5 * d).astype(np.float32)
    d = d.astype(np.float32)
    res = {"scene": args.scene, "rays": n}
    with rtmi.Context(0) as ctx, rtmi.Scene(ctx, g) as sc:
        for rule in (0, 1):
            for _ in range(args.reps):
                tf, hf = rtmi.intersect_method(ctx, sc, o, d, 512.0, rule, rtmi.ISECT_FILTER)
                tm, hm, c = rtmi.intersect_method(ctx, sc, o, d, 512.0, rule, rtmi.ISECT_MFMA, count=True)
            wave = c[: n // 64 * 64].reshape(-1, 64)
            res[f"rule{rule}"] = {"same_hits": bool(np.array_equal(hf, hm)),
                                  "same_t": bool(np.array_equal(tf.view(np.uint32), tm.view(np.uint32))),
                                  "mf_candidates_mean": round(float(c.mean()), 3),
                                  "mf_wave_sum_mean": round(float(wave.sum(axis=1).mean()), 2),
                                  "mf_wave_max_mean": round(float(wave.max(axis=1).mean()), 2)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
