#!/usr/bin/env python3
"""The multi-rank data path with real renders in separate processes, on one GPU.

Run under a launcher, two ranks, both on cuda:0 (RCCL refuses two ranks on one device, so the
collectives run over gloo; RCCL's own gather and all-reduce move the same bytes):

    python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 \\
        --master-port <port> tools/multiproc_gpu_check.py [--out result.json]

Each rank renders its tile set (rtmi.tiles.rank_tiles: 32x32 tiles dealt by diagonals) through
librtmi and rank 0 gathers them (rtmi.dist.FramePipeline, the bench's double-buffered loop);
Expected SARSA runs rtmi.dist.sarsa_frame (each rank renders its tiles, the TD sums are
all-reduced, every rank applies the same update).  Rank 0 then renders the same frames in one
process and checks: the assembled image bit for bit and the ray casts (Cornell, CPU preset), and
for SARSA the images, the ray casts and every rank's Q-table, CDF and visits bit for bit against
the one-process map.  Exit code 0 iff everything matched.
"""
import argparse
import json
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "reinforcement-light-rays-pathtracer_amd"))
import rtmi  # noqa: E402

T = 32


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    dist.init_process_group(backend="gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    res = {"world": world, "backend": "gloo", "device": "cuda:0 for every rank"}
    ok = True
    with rtmi.Context(0) as ctx:
        # ---- the default render (BASELINE config 2's kernel) through the bench's pipeline ----
        geom = rtmi.cornell_geometry(rtmi.RT_PRESET_CPU)
        p = rtmi.default_params(rtmi.RT_PRESET_CPU, width=128, height=96, spp=64, spp_split=64)
        cam = rtmi.camera(rtmi.CAMERAS["cornell"])
        tiles = rtmi.tiles.rank_tiles(p.width, p.height, T, rank, world)
        with rtmi.Scene(ctx, geom) as sc:
            casts = torch.zeros(1, dtype=torch.int64, device=dev)
            stream = torch.cuda.current_stream(dev)

            def render(out):
                rtmi.render_tiles_device(ctx, sc, cam, p, tiles, T, out.data_ptr(), casts.data_ptr(),
                                         stream.cuda_stream)
            pipe = rtmi.dist.FramePipeline(render, (tiles.shape[0], T, T, 3), world, dev)
            for i in range(3):
                pipe.gather_frame(pipe.render_frame(i))
            pipe.drain()
            torch.cuda.synchronize()
            tot = casts.clone()
            dist.all_reduce(tot)  # (per rank: 3 frames)
            if rank == 0:
                img = rtmi.tiles.assemble(pipe.frame(2).cpu().numpy(), p.width, p.height, T, world)
                ref, ref_casts = rtmi.render(ctx, sc, cam, p)
                r = {"bit_exact": bool(np.array_equal(img.view(np.uint32), ref.view(np.uint32))),
                     "ray_casts": int(tot.item()) // 3, "ray_casts_one_process": int(ref_casts)}
                r["ok"] = r["bit_exact"] and r["ray_casts"] == r["ray_casts_one_process"]
                res["render"] = r
                ok = ok and r["ok"]

        # ---- Expected SARSA: tiles + the TD all-reduce (rtmi.dist.sarsa_frame) ----
        g = rtmi.obj_geometry(os.path.join(ROOT, "assets", "models", "door_room.obj"), "door_room")
        ps = rtmi.default_params(rtmi.RT_PRESET_GPU, width=96, height=64, spp=8, spp_split=4)
        cam_d = rtmi.camera(rtmi.CAMERAS["door_room"])
        tiles = rtmi.tiles.rank_tiles(ps.width, ps.height, T, rank, world)
        n_real = rtmi.tiles.rank_tile_count(ps.width, ps.height, T, rank, world)
        frames = 3
        with rtmi.Scene(ctx, g) as sc, rtmi.sarsa.RadianceMap(ctx, sc, 1984) as rm:
            td = rtmi.dist.td_tensors(rm, dev)
            casts = torch.zeros(1, dtype=torch.int64, device=dev)
            out = torch.zeros((tiles.shape[0], T, T, 3), dtype=torch.float32, device=dev)
            imgs, cast_list = [], []
            for _ in range(frames):
                casts.zero_()
                rtmi.dist.sarsa_frame(rm, cam_d, ps, tiles, n_real, T, out, casts, td)
                torch.cuda.synchronize()
                c = casts.clone()
                dist.all_reduce(c)
                cast_list.append(int(c.item()))
                outc = out.cpu()
                glc = [torch.zeros_like(outc) for _ in range(world)] if rank == 0 else None
                dist.gather(outc, gather_list=glc, dst=0)
                if rank == 0:
                    imgs.append(rtmi.tiles.assemble(torch.stack(glc).numpy(), ps.width, ps.height, T, world))
            q, cdf, vis, acc = rm.read()
            # every rank's map must be the same: compare a digest of each rank's state on rank 0
            digest = torch.tensor([int(np.frombuffer(q.tobytes(), np.uint32).astype(np.uint64).sum() % (1 << 62)),
                                   int(vis.astype(np.uint64).sum() % (1 << 62))], dtype=torch.int64)
            digests = [torch.zeros_like(digest) for _ in range(world)] if rank == 0 else None
            dist.gather(digest, gather_list=digests, dst=0)
            if rank == 0:
                with rtmi.sarsa.RadianceMap(ctx, sc, 1984) as one:
                    r = {"frames": frames, "images_bit_exact": [], "ray_casts": cast_list, "ray_casts_one_process": []}
                    for f in range(frames):
                        im, cc = one.render(cam_d, ps, 1)
                        r["images_bit_exact"].append(bool(np.array_equal(im.view(np.uint32),
                                                                          imgs[f].view(np.uint32))))
                        r["ray_casts_one_process"].append(int(cc))
                    q1, cdf1, vis1, acc1 = one.read()
                r["q_cdf_visits_irradiance_bit_exact"] = bool(
                    np.array_equal(q.view(np.uint32), q1.view(np.uint32)) and
                    np.array_equal(cdf.view(np.uint32), cdf1.view(np.uint32)) and
                    np.array_equal(vis, vis1) and np.array_equal(acc.view(np.uint32), acc1.view(np.uint32)))
                r["ranks_same_map"] = all(bool(torch.equal(d, digests[0])) for d in digests)
                r["ok"] = (all(r["images_bit_exact"]) and r["ray_casts"] == r["ray_casts_one_process"]
                           and r["q_cdf_visits_irradiance_bit_exact"] and r["ranks_same_map"])
                res["sarsa"] = r
                ok = ok and r["ok"]
    if rank == 0:
        res["ok"] = ok
        line = json.dumps(res)
        print(line, flush=True)
        if args.out:
            with open(args.out, "w") as f:
                f.write(line + "\n")
    flag = torch.tensor([1 if ok else 0], dtype=torch.int64)
    dist.broadcast(flag, 0)
    dist.destroy_process_group()
    sys.exit(0 if int(flag.item()) == 1 else 1)


if __name__ == "__main__":
    main()
