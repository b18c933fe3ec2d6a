"""Multi-GPU frame assembly: one process per GPU, image tiles dealt to the
ranks by diagonals (rtmi.tiles: tile (tx, ty) -> rank (tx + ty) mod P), one gather of the
equal-sized per-rank tile buffers to rank 0 over RCCL (backend "nccl" on ROCm: ncclSend /
ncclRecv pairs; "gloo" for CPU tests).  Only rank 0 consumes the frame (the SDL frame
buffer of the reference's loop), so the other ranks receive nothing: an all-gather would
move P times the bytes (2048^2 on 8 GPUs: 44 MB into every rank instead of 6.3 MB per
rank into one).

Data path per frame: rank r renders its tiles
into out[k, T, T, 3] -> gather(dst=0) -> gathered[P, k, T, T, 3] on rank 0
-> rtmi.tiles.assemble.  Message per rank = k*T*T*12 B (512^2 frame on 8 GPUs: 393 KB).
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def gather_tiles(out: torch.Tensor, gathered, async_op: bool = False, dst: int = 0):
    """Gather the per-rank tile buffers (out: [k, T, T, 3]) into gathered: [world, k, T, T, 3]
    on rank `dst` (other ranks pass gathered = None and receive nothing).  async_op: return
    the collective's work handle (RCCL runs on its own stream after the work already queued
    on the current one; work.wait() makes the current stream wait for it) so the next
    frame's render overlaps the exchange; None when there is nothing to wait for."""
    world = dist.get_world_size() if dist.is_initialized() else 1
    if world == 1:
        gathered[0].copy_(out)
        return None if async_op else gathered
    root = dist.get_rank() == dst
    glist = list(gathered.unbind(0)) if root else None
    work = dist.gather(out, gather_list=glist, dst=dst, async_op=async_op)
    return work if async_op else gathered


class FramePipeline:
    """Two frame buffers per rank: frame i renders into buffer i % 2 while frame i-1
    is gathered to rank 0 from the other one (bench.py).  `render(out)` queues one frame's
    render into `out` ([k, T, T, 3]) on the current stream; a buffer is rendered into
    again only after its previous gather completed (work.wait() orders the current
    stream after the collective -- a host wait on gloo)."""

    def __init__(self, render, shape, world: int, device):
        self.render = render
        self.world = world
        self.outs = [torch.zeros(shape, dtype=torch.float32, device=device) for _ in range(2)]
        self.root = world == 1 or dist.get_rank() == 0
        # the assembled frames live on rank 0 only
        self.gathered = [torch.empty((world,) + tuple(shape), dtype=torch.float32, device=device)
                         if self.root and world > 1 else None for _ in range(2)]
        self.pending = [None, None]

    def wait(self, b: int) -> None:
        if self.pending[b] is not None:
            self.pending[b].wait()
            self.pending[b] = None

    def render_frame(self, i: int) -> int:
        b = i % 2
        self.wait(b)
        self.render(self.outs[b])
        return b

    def gather_frame(self, b: int) -> None:
        if self.world > 1:
            self.pending[b] = gather_tiles(self.outs[b], self.gathered[b], async_op=True)

    def drain(self) -> None:
        for b in range(2):
            self.wait(b)

    def frame(self, i: int) -> torch.Tensor:
        """[world, k, T, T, 3] tiles of frame i on rank 0 (after drain(), for the last two
        frames); None on the other ranks."""
        b = i % 2
        return self.outs[b][None] if self.world == 1 else self.gathered[b]


def sum_td(td_sum: torch.Tensor, td_count: torch.Tensor) -> None:
    """Expected-SARSA frame exchange: sum every rank's TD accumulators in place
    (int64 fixed-point target sums and int32 visit counts, [n_volumes*144]).
    Integer sums are exact and order-free, so the Q-table every rank applies is
    bit-identical to the single-GPU one for any world size."""
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(td_sum, op=dist.ReduceOp.SUM)
        dist.all_reduce(td_count, op=dist.ReduceOp.SUM)


class _DevArray:
    """__cuda_array_interface__ view of a device buffer owned by librtmi."""

    def __init__(self, ptr: int, n: int, typestr: str):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": typestr, "data": (ptr, False),
                                         "version": 3, "strides": None}


def td_tensors(radiance_map, device: torch.device):
    """torch views (no copy) of a RadianceMap's device TD accumulators."""
    s, c, n = radiance_map.td_device()
    ts = torch.as_tensor(_DevArray(s, n, "<i8"), device=device)
    tc = torch.as_tensor(_DevArray(c, n, "<i4"), device=device)
    return ts, tc


def sarsa_frame(radiance_map, cam, params, tiles, n_real: int, tile_size: int, out: torch.Tensor,
                casts: torch.Tensor, td=None) -> None:
    """One multi-GPU SARSA frame: render this rank's n_real real tiles (the padding slots
    of `tiles` are left untouched so no pixel is learned from twice; TD sums stay in the
    map), all-reduce the TD sums over ranks, apply the shared update on every rank."""
    world = dist.get_world_size() if dist.is_initialized() else 1
    if world > 1 and getattr(radiance_map, "td_mode", 0) != 0:
        raise ValueError("the in-frame TD mode updates one GPU's map in place: no TD sums to share")
    stream = torch.cuda.current_stream(out.device).cuda_stream
    radiance_map.render_tiles_device(cam, params, tiles[:n_real], tile_size, out.data_ptr(), casts.data_ptr(),
                                     apply=(world == 1), stream=stream)
    if world > 1:
        ts, tc = td if td is not None else td_tensors(radiance_map, out.device)
        sum_td(ts, tc)
        radiance_map.apply(stream)
