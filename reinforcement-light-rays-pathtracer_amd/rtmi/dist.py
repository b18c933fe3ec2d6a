"""Multi-GPU frame assembly: one process per GPU, image tiles round-robin
over ranks (rtmi.tiles), one all-gather of the equal-sized per-rank tile
buffers over RCCL (backend "nccl" on ROCm; "gloo" for CPU tests).

Data path per frame: rank r renders tiles k = r, r+P, ...
into out[k_r, T, T, 3] -> all_gather_into_tensor -> gathered[P, k_r, T, T, 3]
-> rtmi.tiles.assemble on the consumer.  Message per rank = k_r*T*T*12 B
(512^2 frame on 8 GPUs: 393 KB per rank).
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def gather_tiles(out: torch.Tensor, gathered: torch.Tensor) -> torch.Tensor:
    """All-gather the per-rank tile buffers (out: [k, T, T, 3]) into
    gathered: [world, k, T, T, 3]."""
    world = dist.get_world_size() if dist.is_initialized() else 1
    if world == 1:
        gathered[0].copy_(out)
        return gathered
    dist.all_gather_into_tensor(gathered.view(world * out.shape[0], *out.shape[1:]), out)
    return gathered
