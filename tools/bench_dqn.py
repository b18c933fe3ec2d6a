#!/usr/bin/env python3
"""DQN path measurements (BASELINE config 4): the MFMA forward alone and the
full wavefront render.

    python tools/bench_dqn.py [--rays 1048576] [--width 1024] [--spp 1] [--scene archway]

Prints one JSON line: MLP TFLOP/s against the bf16 dense MFMA peak (2.5 PF),
render ms per sample and Mrays/s.
"""
import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "reinforcement-light-rays-pathtracer_amd"))
import rtmi  # noqa: E402

MFMA_BF16_PEAK_TFLOPS = 2500.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="archway")
    ap.add_argument("--rays", type=int, default=1 << 20)
    ap.add_argument("--width", type=int, default=1024)
    ap.add_argument("--spp", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--max-bounces", type=int, default=80)
    ap.add_argument("--no-render", action="store_true", help="forward pass only (profiling)")
    ap.add_argument("--mlp", default="stream", choices=["stream", "stationary"],
                    help="forward kernel: weight-streaming (default) or weight-stationary")
    args = ap.parse_args()
    g = rtmi.obj_geometry(os.path.join(ROOT, "assets", "models", args.scene + ".obj"), args.scene)
    if args.scene == "door_room":
        W, b = rtmi.dqn.split_layers(rtmi.dqn.read_dynet(os.path.join(ROOT, "assets", "models",
                                                                        "door_room_12_12.model")))
        weights = "trained door_room_12_12.model"
    else:
        W, b = rtmi.dqn.synthetic_weights(g.nn_vertices.size)
        weights = "synthetic He-normal seed 1984"
    ctx = rtmi.Context(0)
    sc = rtmi.Scene(ctx, g)
    net = rtmi.dqn.Dqn(ctx, g.nn_vertices, W, b)
    net.set_mlp(net.MLP_STATIONARY if args.mlp == "stationary" else net.MLP_STREAM)
    stream = torch.cuda.current_stream()
    res = {"scene": args.scene, "weights": weights, "n_in": int(g.nn_vertices.size), "mlp_kernel": args.mlp}

    # --- forward alone: random positions in the scene's bounding box
    lo, hi = g.all_triangles().reshape(-1, 3).min(0), g.all_triangles().reshape(-1, 3).max(0)
    loc = torch.from_numpy((lo + (hi - lo) * np.random.default_rng(0).random((args.rays, 3))).astype(np.float32)).cuda()
    q = torch.empty((args.rays, 144), dtype=torch.float32, device="cuda")
    for _ in range(2):
        net.forward_device(loc.data_ptr(), args.rays, q.data_ptr(), stream.cuda_stream)
    torch.cuda.synchronize()
    ts = []
    for _ in range(10):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        net.forward_device(loc.data_ptr(), args.rays, q.data_ptr(), stream.cuda_stream)
        e1.record(stream)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ms = float(np.median(ts))
    tflops = net.flops_per_ray() * args.rays / (ms * 1e-3) / 1e12
    res["mlp"] = {"rays": args.rays, "ms": round(ms, 4), "tflops": round(tflops, 2),
                  "frac_bf16_peak": round(tflops / MFMA_BF16_PEAK_TFLOPS, 4),
                  "flops_per_ray": net.flops_per_ray(),
                  # what the MFMA units actually execute (layers 1-3; layer 0 is folded)
                  "mfma_flops_per_ray": net.mfma_flops_per_ray(),
                  "mfma_tflops": round(net.mfma_flops_per_ray() * args.rays / (ms * 1e-3) / 1e12, 2),
                  "q_mean": float(q.mean().item())}

    if args.no_render:
        print(json.dumps(res), flush=True)
        return
    # --- full render: one frame of `spp` samples per step
    p = rtmi.default_params(rtmi.RT_PRESET_GPU, width=args.width, height=args.width, spp=args.spp,
                            max_bounces=args.max_bounces)
    cam = rtmi.camera(rtmi.CAMERAS[args.scene])
    tiles = rtmi.tiles.tile_origins(args.width, args.width, 32)
    out = torch.zeros((len(tiles), 32, 32, 3), dtype=torch.float32, device="cuda")
    casts = torch.zeros(1, dtype=torch.int64, device="cuda")
    rtmi.dqn.render_tiles_device(ctx, sc, net, cam, p, tiles, 32, out.data_ptr(), casts.data_ptr(),
                                 stream.cuda_stream)
    torch.cuda.synchronize()
    casts.zero_()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        rtmi.dqn.render_tiles_device(ctx, sc, net, cam, p, tiles, 32, out.data_ptr(), casts.data_ptr(),
                                     stream.cuda_stream)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    c = int(casts.item())
    res["render"] = {"width": args.width, "spp_per_step": args.spp, "steps": args.steps,
                     "ms_per_step": round(dt / args.steps * 1e3, 2), "ray_casts": c,
                     "mrays_s": round(c / dt / 1e6, 2),
                     "casts_per_sample_per_pixel": round(c / (args.steps * args.spp * args.width ** 2), 3),
                     "image_mean": float(out.mean().item()),
                     "image_sha1": hashlib.sha1(out.cpu().numpy().tobytes()).hexdigest()[:16]}
    print(json.dumps(res), flush=True)
    net.close()
    sc.close()
    ctx.close()


if __name__ == "__main__":
    main()
