"""Row-interleaved frame sharding over ranks + one gather to rank 0.

Pixels are independent and each pixel's RNG subsequence is its GLOBAL index, so a frame splits by
rows with no exchange during rendering; the only collective is one gather of each shard's rows to
rank 0 at the end of the frame (RCCL over xGMI with the "nccl" backend on GPUs, gloo in the CPU tests),
followed by a row un-permute on rank 0.  gather_rows moves whatever dtype it is given: bench.py gathers
the u8 PPM bytes the render kernel writes (3 B/pixel), the tests gather float32 frames too.  This is not a translation of any reference
collective: the reference is single-GPU.
"""
from __future__ import annotations

import math

import torch
import torch.distributed as dist

from . import shard_rows


def weak_scaled_resolution(width: int, height: int, world: int) -> tuple[int, int]:
    """Frame for weak scaling: ~world x the pixels of (width, height) at the same aspect and camera,
    so every rank keeps ~width*height pixels of the same scene content."""
    if world <= 1:
        return width, height
    s = math.sqrt(world)
    return int(round(width * s)), int(round(height * s))


def max_shard_rows(height: int, world: int) -> int:
    return (height + world - 1) // world


def gather_rows(local: torch.Tensor, height: int, width: int, rank: int, world: int,
                group=None) -> torch.Tensor | None:
    """Gather row-interleaved shards [rows_r, W, 3] onto rank 0 and assemble [H, W, 3].

    Shards are padded to ceil(H/world) rows so one fixed-size gather moves everything
    (per-rank message = ceil(H/G) * W * 3 * itemsize bytes: 0.78 MB of u8 PPM bytes at 1080p/8 GPUs,
    3.1 MB of float32)."""
    rows = max_shard_rows(height, world)
    if local.shape[0] != rows:
        pad = torch.zeros((rows - local.shape[0], width, 3), dtype=local.dtype, device=local.device)
        local = torch.cat([local, pad], dim=0)
    if world == 1:
        return local[:height]
    bufs = [torch.empty_like(local) for _ in range(world)] if rank == 0 else None
    dist.gather(local.contiguous(), gather_list=bufs, dst=0, group=group)
    if rank != 0:
        return None
    img = torch.empty((height, width, 3), dtype=local.dtype, device=local.device)
    for r in range(world):
        _, _, cnt = shard_rows(height, r, world)
        img[r::world] = bufs[r][:cnt]
    return img
