#!/usr/bin/env python3
"""One measurement per BASELINE.json config on ONE MI355X (device-buffer paths,
HIP events on the launch stream), written as one JSON document.

    python tools/bench_configs.py [--out gpurun_out/configs.json] [--only c2 c3 ...]

  c1  Cornell 256^2, 4 spp, CPU-engine preset: GPU frame vs the CPU restatement
      (oracle/, OpenMP, this host) on the same frame; images compared bit for bit.
  c2  Cornell 512^2, 256 spp (bench.py's workload): one frame.
  c3  door_room 512^2, 256 spp, Expected SARSA: frames 0..2 (the Q-table learns
      between frames; paths shorten).
  c4  archway 1024^2, DQN Q-weighted sampling (fc_layer MFMA forward), synthetic
      He-normal weights (the archway model is not in the reference): `--dqn-spp`
      samples of the 512-spp config (Mrays/s is per-sample-count independent).
  c5  complex_light_room 2048^2, 8-GPU tile split: the tile set of every rank r of
      P = 8 rendered alone on this GPU at `--c5-spp` samples: max_r is the kernel
      part of one 8-GPU frame, the sum the 1-GPU frame.
  cpu the CPU restatement's ray-cast rate on bounded samples of c3-c5 (this host).
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "reinforcement-light-rays-pathtracer_amd"))
import rtmi  # noqa: E402

MODELS = os.path.join(ROOT, "assets", "models")
TILE = 32


def timed(fn, stream):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    fn()
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1)


def tile_render(ctx, sc, cam, p, tiles, stream, repeat=1):
    out = torch.zeros((len(tiles), TILE, TILE, 3), dtype=torch.float32, device="cuda")
    casts = torch.zeros(1, dtype=torch.int64, device="cuda")
    fn = lambda: rtmi.render_tiles_device(ctx, sc, cam, p, tiles, TILE, out.data_ptr(), casts.data_ptr(),
                                          stream.cuda_stream)
    fn()
    torch.cuda.synchronize()
    ms = []
    for _ in range(repeat):
        casts.zero_()
        ms.append(timed(fn, stream))
    return float(np.median(ms)), int(casts.item()), out


def c1(ctx, stream):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # the CPU restatement: checker and CPU baseline only
    g = rtmi.cornell_geometry(rtmi.RT_PRESET_CPU)
    p = rtmi.default_params(rtmi.RT_PRESET_CPU, width=256, height=256, spp=4, spp_split=4)
    with rtmi.Scene(ctx, g) as sc:
        tiles = rtmi.tiles.tile_origins(256, 256, TILE)
        ms, casts, out = tile_render(ctx, sc, rtmi.camera(rtmi.CAMERAS["cornell"]), p, tiles, stream, 5)
        img = rtmi.tiles.assemble(out.cpu().numpy()[None], 256, 256, TILE, 1)
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or os.cpu_count() or 1
    oracle.set_threads(threads)
    t0 = time.perf_counter()
    ref, rc = oracle.render(g, oracle.camera(rtmi.CAMERAS["cornell"]), oracle.params_from(p))
    cpu_s = time.perf_counter() - t0
    return {"gpu_ms": round(ms, 4), "ray_casts": casts, "gpu_mrays_s": round(casts / ms / 1e3, 1),
            "cpu_ms": round(cpu_s * 1e3, 2), "cpu_threads": threads, "cpu_mrays_s": round(rc / cpu_s / 1e6, 2),
            "bit_exact_vs_cpu": bool(np.array_equal(img.view(np.uint32), ref.view(np.uint32)) and rc == casts)}


def c2(ctx, stream):
    g = rtmi.cornell_geometry(rtmi.RT_PRESET_CPU)
    # bench.py's split (64 lanes per pixel, 4 samples each): at 32 the sample slots of
    # k_render_ps exceed its LDS budget and the frame falls back to k_render
    p = rtmi.default_params(rtmi.RT_PRESET_CPU, width=512, height=512, spp=256, spp_split=64)
    with rtmi.Scene(ctx, g) as sc:
        tiles = rtmi.tiles.tile_origins(512, 512, TILE)
        ms, casts, _ = tile_render(ctx, sc, rtmi.camera(rtmi.CAMERAS["cornell"]), p, tiles, stream, 5)
    return {"frame_ms": round(ms, 4), "ray_casts": casts, "mrays_s": round(casts / ms / 1e3, 1)}


def c3(ctx, stream, frames):
    g = rtmi.obj_geometry(os.path.join(MODELS, "door_room.obj"), "door_room")
    p = rtmi.default_params(rtmi.RT_PRESET_GPU, width=512, height=512, spp=256, spp_split=8)
    cam = rtmi.camera(rtmi.CAMERAS["door_room"])
    res = []
    with rtmi.Scene(ctx, g) as sc:
        rm = rtmi.sarsa.RadianceMap(ctx, sc, 1984)
        tiles = rtmi.tiles.tile_origins(512, 512, TILE)
        out = torch.zeros((len(tiles), TILE, TILE, 3), dtype=torch.float32, device="cuda")
        casts = torch.zeros(1, dtype=torch.int64, device="cuda")
        for f in range(frames):
            casts.zero_()
            ms = timed(lambda: rm.render_tiles_device(cam, p, tiles, TILE, out.data_ptr(), casts.data_ptr(), True,
                                                      stream.cuda_stream), stream)
            c = int(casts.item())
            res.append({"frame": f, "ms": round(ms, 2), "mrays_s": round(c / ms / 1e3, 1),
                        "avg_path_length": round(c / (512 * 512 * 256), 3)})
        stats = rm.search_stats()
        n_vol = rm.n_volumes
        rm.close()
    return {"volumes": n_vol, "frames": res, "search": stats}


def c4(ctx, stream, spp):
    g = rtmi.obj_geometry(os.path.join(MODELS, "archway.obj"), "archway")
    W, b = rtmi.dqn.synthetic_weights(g.nn_vertices.size)
    p = rtmi.default_params(rtmi.RT_PRESET_GPU, width=1024, height=1024, spp=spp)
    cam = rtmi.camera(rtmi.CAMERAS["archway"])
    with rtmi.Scene(ctx, g) as sc, rtmi.dqn.Dqn(ctx, g.nn_vertices, W, b) as net:
        tiles = rtmi.tiles.tile_origins(1024, 1024, TILE)
        out = torch.zeros((len(tiles), TILE, TILE, 3), dtype=torch.float32, device="cuda")
        casts = torch.zeros(1, dtype=torch.int64, device="cuda")
        fn = lambda: rtmi.dqn.render_tiles_device(ctx, sc, net, cam, p, tiles, TILE, out.data_ptr(),
                                                  casts.data_ptr(), stream.cuda_stream)
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3  # includes the host's every-4-bounce list checks
        c = int(casts.item())
    return {"spp": spp, "ms": round(ms, 1), "ray_casts": c, "mrays_s": round(c / ms / 1e3, 1),
            "ms_512spp_extrapolated": round(ms * 512 / spp, 0), "weights": "synthetic He-normal seed 1984"}


def c5(ctx, stream, spp, world=8, split=8):
    g = rtmi.obj_geometry(os.path.join(MODELS, "complex_light_room.obj"), "complex_light_room")
    p = rtmi.default_params(rtmi.RT_PRESET_GPU, width=2048, height=2048, spp=spp, spp_split=split)
    cam = rtmi.camera(rtmi.CAMERAS["complex_light_room"])
    per = []
    tot = 0
    with rtmi.Scene(ctx, g) as sc:
        for r in range(world):
            tiles = rtmi.tiles.rank_tiles(2048, 2048, TILE, r, world)[:rtmi.tiles.rank_tile_count(2048, 2048, TILE, r,
                                                                                                     world)]
            ms, casts, _ = tile_render(ctx, sc, cam, p, tiles, stream, 1)
            per.append(round(ms, 2))
            tot += casts
    return {"spp": spp, "spp_split": split, "ranks": world, "ms_per_rank": per, "ms_8gpu_kernel": max(per),
            "ms_1gpu": round(sum(per), 2), "kernel_speedup_8": round(sum(per) / max(per), 3),
            "ray_casts": tot, "mrays_s_1gpu": round(tot / sum(per) / 1e3, 1),
            "ms_1024spp_8gpu_extrapolated": round(max(per) * 1024 / spp, 0)}


def cpu_configs(which):
    """The CPU restatement (oracle/, OpenMP over rows, this host's cores) on a bounded sample
    of configs 3-5: ray casts per second, to set beside the GPU's.  Per-sample cost does not
    depend on spp within a frame, so a few spp stand for the configs' 256/512/1024."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # the CPU restatement: CPU baseline only
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or os.cpu_count() or 1
    oracle.set_threads(threads)
    out = {}
    if "c3" in which:  # frame 0 of Expected SARSA (TD accumulation and the end-of-frame update)
        g = rtmi.obj_geometry(os.path.join(MODELS, "door_room.obj"), "door_room")
        m = oracle.Sarsa(g, 1984)
        p = rtmi.default_params(rtmi.RT_PRESET_GPU, width=512, height=512, spp=2)
        t0 = time.perf_counter()
        _, c = m.render(oracle.camera(rtmi.CAMERAS["door_room"]), oracle.params_from(p), 1)
        dt = time.perf_counter() - t0
        out["c3"] = {"sample": "door_room 512^2 x 2 spp, frame 0", "ray_casts": c, "s": round(dt, 2),
                     "cpu_mrays_s": round(c / dt / 1e6, 2), "threads": threads}
    if "c4" in which:  # DQN sampling with the bf16-emulating forward (prepared weights)
        g = rtmi.obj_geometry(os.path.join(MODELS, "archway.obj"), "archway")
        W, b = rtmi.dqn.synthetic_weights(g.nn_vertices.size)
        p = rtmi.default_params(rtmi.RT_PRESET_GPU, width=1024, height=1024, spp=1)
        t0 = time.perf_counter()
        _, c = oracle.render_dqn(g, W, b, g.nn_vertices, oracle.camera(rtmi.CAMERAS["archway"]),
                                 oracle.params_from(p), (448, 448, 64, 64), bf16=True)
        dt = time.perf_counter() - t0
        out["c4"] = {"sample": "archway 1024^2 window 64^2 at (448, 448) x 1 spp", "ray_casts": c,
                     "s": round(dt, 2), "cpu_mrays_s": round(c / dt / 1e6, 3), "threads": threads}
    if "c5" in which:
        g = rtmi.obj_geometry(os.path.join(MODELS, "complex_light_room.obj"), "complex_light_room")
        p = rtmi.default_params(rtmi.RT_PRESET_GPU, width=2048, height=2048, spp=4)
        t0 = time.perf_counter()
        _, c = oracle.render(g, oracle.camera(rtmi.CAMERAS["complex_light_room"]), oracle.params_from(p),
                             (0, 1008, 2048, 32))
        dt = time.perf_counter() - t0
        out["c5"] = {"sample": "complex_light_room 2048^2 rows 1008..1039 x 4 spp", "ray_casts": c,
                     "s": round(dt, 2), "cpu_mrays_s": round(c / dt / 1e6, 2), "threads": threads}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "configs.json"))
    ap.add_argument("--sarsa-frames", type=int, default=3)
    ap.add_argument("--dqn-spp", type=int, default=16)
    ap.add_argument("--c5-spp", type=int, default=64)
    ap.add_argument("--c5-split", type=int, default=32)  # bench.py's config-5 split
    ap.add_argument("--only", nargs="*", default=None)
    ap.add_argument("--cpu", nargs="*", default=["c3", "c4", "c5"],
                    help="configs whose CPU-restatement rate to measure (empty: none)")
    args = ap.parse_args()
    stream = torch.cuda.current_stream()
    res = {"device": torch.cuda.get_device_name(0)}
    with rtmi.Context(0) as ctx:
        steps = {"c1": lambda: c1(ctx, stream), "c2": lambda: c2(ctx, stream),
                 "c3": lambda: c3(ctx, stream, args.sarsa_frames), "c4": lambda: c4(ctx, stream, args.dqn_spp),
                 "c5": lambda: c5(ctx, stream, args.c5_spp, split=args.c5_split)}
        for k, fn in steps.items():
            if args.only and k not in args.only:
                continue
            res[k] = fn()
            print(k, json.dumps(res[k]), flush=True)
    if args.cpu:
        res["cpu"] = cpu_configs(args.cpu)
        print("cpu", json.dumps(res["cpu"]), flush=True)
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as fh:
        json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
