"""Instrumentation of the two SARSA TD rules on config 3's scene.

door_room, 64^2 x 16 spp (spp_split 4), frame 0 then frames 1-3, per seed:
  * the restatement's frame-synchronous rule (oracle mode 0, = the GPU default bit for bit)
    and its sequential in-frame rule (oracle mode 1: the reference's update applied event by
    event in the render's order);
  * with --gpu, the GPU's in-frame mode (racy, every lane) and its default mode;
  * per frame: image mean, paired z of the per-pixel difference against the restatement's
    in-frame frame, the restatement's CDF-sample statistics (samples, failed samples -- the
    reference's null ray --, samples that took sector 0).

    python3 tools/sarsa_inframe_probe.py [--gpu] [--seeds 1984 7 11 13] --out <json>
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "reinforcement-light-rays-pathtracer_amd"), os.path.join(ROOT, "oracle")]

import oracle  # noqa: E402  (the checker)
import rtmi  # noqa: E402


def paired_z(a, b):
    d = (a.mean(axis=2) - b.mean(axis=2)).ravel().astype(np.float64)
    return float(d.mean() / (d.std(ddof=1) / np.sqrt(d.size)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpu", action="store_true")
    ap.add_argument("--seeds", type=int, nargs="+", default=[1984, 7, 11, 13])
    ap.add_argument("--frames", type=int, default=3)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    g = rtmi.obj_geometry(os.path.join(ROOT, "assets", "models", "door_room.obj"), "door_room")
    cam = rtmi.camera(rtmi.CAMERAS["door_room"])
    ocam = oracle.camera(rtmi.CAMERAS["door_room"])
    ctx = sc = None
    if args.gpu:
        ctx = rtmi.Context(0)
        sc = rtmi.Scene(ctx, g)
    res = {"scene": "door_room", "width": 64, "height": 64, "spp": 16, "spp_split": 4, "seeds": {}}
    t0 = time.time()
    for seed in args.seeds:
        # the seed keys both the volume placement and the path RNG (Philox key)
        p = rtmi.default_params(rtmi.RT_PRESET_GPU, width=64, height=64, spp=16, spp_split=4, seed=seed)
        op = oracle.params_from(p)
        maps = {"oracle_frame": oracle.Sarsa(g, seed), "oracle_inframe": oracle.Sarsa(g, seed)}
        maps["oracle_inframe"].set_td_mode(1)
        if args.gpu:
            maps["gpu_frame"] = rtmi.sarsa.RadianceMap(ctx, sc, seed)
            maps["gpu_inframe"] = rtmi.sarsa.RadianceMap(ctx, sc, seed)
            maps["gpu_inframe"].set_td_mode(rtmi.sarsa.TD_INFRAME)
        out = {k: {"mean": [], "z_vs_oracle_inframe": []} for k in maps}
        for k in ("oracle_frame", "oracle_inframe"):
            out[k].update(cdf_samples=[], null_samples=[], sector0=[])
        for f in range(1 + args.frames):
            imgs = {}
            for k, m in maps.items():
                if k.startswith("gpu"):
                    imgs[k] = m.render(cam, p, 1)[0]
                else:
                    imgs[k] = m.render(ocam, op, 1)[0]
                    c, n, s0 = m.sample_stats()
                    out[k]["cdf_samples"].append(c)
                    out[k]["null_samples"].append(n)
                    out[k]["sector0"].append(s0)
            for k in maps:
                out[k]["mean"].append(float(imgs[k].mean()))
                same = np.array_equal(imgs[k], imgs["oracle_inframe"])
                out[k]["z_vs_oracle_inframe"].append(0.0 if same else paired_z(imgs[k], imgs["oracle_inframe"]))
            print(f"seed {seed} frame {f}: " + " ".join(f"{k} {out[k]['mean'][-1]:.4f} "
                                                        f"(z {out[k]['z_vs_oracle_inframe'][-1]:+.2f})"
                                                        for k in maps), f"[{time.time() - t0:.0f} s]", flush=True)
        for k, m in maps.items():
            zs = out[k]["z_vs_oracle_inframe"][1:]
            out[k]["z_combined_frames_1_on"] = float(sum(zs) / np.sqrt(len(zs)))
            if k.startswith("gpu"):
                m.close()
        res["seeds"][str(seed)] = out
    if sc is not None:
        sc.close()
        ctx.close()
    if args.out:
        with open(args.out, "w") as fh:
            json.dump(res, fh, indent=1)
    print(json.dumps({s: {k: v["z_combined_frames_1_on"] for k, v in o.items()} for s, o in res["seeds"].items()}))


if __name__ == "__main__":
    main()
