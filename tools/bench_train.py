#!/usr/bin/env python3
"""Neural-Q training step measurements (rt_dqn_train_step_device).

    python tools/bench_train.py [--scene archway] [--batch 4096 65536] [--steps 20]

One step = forward with activations kept, loss, backward, clipping and Adam over all
parameters, on `batch` rays (the reference trains in batches of ray_batch_size).  Prints
one JSON line per batch: ms per step (HIP events on the launch stream), rays/s, and the
step's rate in the reference's algorithmic flops (forward 2*sum(in*out) per ray, backward
dW the same, dX the same minus layer 0) against the 157.3 TF/s fp32 peak; and the flops
the MFMA GEMMs execute (layer 0 is folded: layers 1-3 forward, dW, dX).
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "reinforcement-light-rays-pathtracer_amd"))
import rtmi  # noqa: E402

FP32_PEAK_TFLOPS = 157.3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="archway")
    ap.add_argument("--batch", type=int, nargs="*", default=[4096, 65536])
    ap.add_argument("--steps", type=int, default=20)
    args = ap.parse_args()
    g = rtmi.obj_geometry(os.path.join(ROOT, "assets", "models", args.scene + ".obj"), args.scene)
    W, b = rtmi.dqn.synthetic_weights(g.nn_vertices.size)
    dims = [W[0].shape[1]] + [w.shape[0] for w in W]
    mac = sum(dims[i] * dims[i + 1] for i in range(4))
    # the reference's step (DyNet: explicit n_in-wide layer 0): forward, dW, dX (no dX of layer 0)
    flops_per_ray = 2 * mac * 3 - 2 * dims[0] * dims[1]
    # what the GEMMs of this step execute: layer 0 is folded (no n_in-wide GEMM at all)
    mac_gemm = sum(dims[i] * dims[i + 1] for i in range(1, 4))
    gemm_flops_per_ray = 2 * mac_gemm * 3
    ctx = rtmi.Context(0)
    stream = torch.cuda.current_stream()
    rng = np.random.default_rng(0)
    lo, hi = g.all_triangles().reshape(-1, 3).min(0), g.all_triangles().reshape(-1, 3).max(0)
    for n in args.batch:
        loc = torch.from_numpy((lo + (hi - lo) * rng.random((n, 3))).astype(np.float32)).cuda()
        act = torch.from_numpy(rng.integers(0, 144, n).astype(np.int32)).cuda()
        tgt = torch.from_numpy(rng.uniform(0.5, 1.5, n).astype(np.float32)).cuda()
        with rtmi.dqn.DqnTrainer(ctx, g.nn_vertices, W, b) as tr:
            first = tr.step_device(loc.data_ptr(), act.data_ptr(), tgt.data_ptr(), n, stream.cuda_stream)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(args.steps):
                tr.step_device(loc.data_ptr(), act.data_ptr(), tgt.data_ptr(), n, stream.cuda_stream, sync=False)
            e1.record(stream)
            torch.cuda.synchronize()
            last = tr.step_device(loc.data_ptr(), act.data_ptr(), tgt.data_ptr(), n, stream.cuda_stream)
        ms = e0.elapsed_time(e1) / args.steps
        tf = flops_per_ray * n / (ms * 1e-3) / 1e12
        print(json.dumps({"scene": args.scene, "dims": dims, "batch": n, "ms_per_step": round(ms, 4),
                          "rays_per_s": round(n / (ms * 1e-3), 1), "flops_per_ray": flops_per_ray,
                          "tflops": round(tf, 2), "frac_fp32_peak": round(tf / FP32_PEAK_TFLOPS, 4),
                          "gemm_flops_per_ray": gemm_flops_per_ray,
                          "gemm_tflops_executed": round(gemm_flops_per_ray * n / (ms * 1e-3) / 1e12, 2),
                          "loss_first": first[0], "loss_last": last[0]}), flush=True)


if __name__ == "__main__":
    main()
