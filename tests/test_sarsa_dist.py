"""Multi-rank Expected-SARSA frame exchange (CPU, gloo, world 2).

Each rank renders its tiles of a frame; the frame's TD accumulators (int64 fixed-point
target sums and int32 visit counts per (volume, sector), the device layout of
rt_sarsa_td_device) are then summed over the ranks with rtmi.dist.sum_td, and every rank
applies the same update.  The accumulators here are real ones: the CPU restatement's TD
sums of each rank's tiles of a Cornell frame (oracle.Sarsa.td_rect), reference semantics
of temporal_difference_update (GPU/radiance_volumes/radiance_volume.cu:282-301).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

W = H = 64
TILE = 32


def _rank_td(oracle_mod, rtmi_mod, smap, ocam, op, rank, world):
    tiles = rtmi_mod.tiles.rank_tiles(W, H, TILE, rank, world)
    n = rtmi_mod.tiles.rank_tile_count(W, H, TILE, rank, world)
    s_tot, c_tot = None, None
    for (x, y) in tiles[:n]:
        s, c = smap.td_rect(ocam, op, (int(x), int(y), TILE, TILE))
        s_tot = s if s_tot is None else s_tot + s
        c_tot = c if c_tot is None else c_tot + c
    return s_tot, c_tot.astype(np.int32)


def _worker(rank, world, port, s, c, want_s, want_c, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "reinforcement-light-rays-pathtracer_amd"))
    import rtmi
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ts = torch.from_numpy(s.copy())
    tc = torch.from_numpy(c.copy())
    rtmi.dist.sum_td(ts, tc)
    q.put((rank, bool(np.array_equal(ts.numpy(), want_s) and np.array_equal(tc.numpy(), want_c))))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    so = socket.socket()
    so.bind(("127.0.0.1", 0))
    p = so.getsockname()[1]
    so.close()
    return p


def test_gloo_world2_td_exchange_equals_single_rank(rtmi_mod, oracle_mod):
    geom = rtmi_mod.cornell_geometry(rtmi_mod.RT_PRESET_GPU)
    smap = oracle_mod.Sarsa(geom, 1984)
    p = rtmi_mod.default_params(rtmi_mod.RT_PRESET_GPU, width=W, height=H, spp=2, max_bounces=8)
    op = oracle_mod.params_from(p)
    ocam = oracle_mod.camera(rtmi_mod.CAMERAS["cornell"])
    full_s, full_c = smap.td_rect(ocam, op, (0, 0, W, H))
    full_c = full_c.astype(np.int32)
    parts = [_rank_td(oracle_mod, rtmi_mod, smap, ocam, op, r, 2) for r in range(2)]
    assert full_c.sum() > 0 and np.count_nonzero(parts[0][1]) and np.count_nonzero(parts[1][1])
    # the ranks' accumulators differ (different tiles) and add up to the frame's
    assert not np.array_equal(parts[0][1], parts[1][1])
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, parts[r][0], parts[r][1], full_s, full_c, q))
             for r in range(2)]
    for pr in procs:
        pr.start()
    res = dict(q.get(timeout=120) for _ in range(2))
    for pr in procs:
        pr.join(timeout=60)
    assert all(pr.exitcode == 0 for pr in procs)
    assert res == {0: True, 1: True}
