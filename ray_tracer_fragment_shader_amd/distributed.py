"""Image-space data parallelism across the GPUs of one node.

One process per GPU.  A frame's rows are cut into bands of `band_height` rows dealt round-robin to the
ranks (rt_rows); contiguous stripes would be badly imbalanced (sky rows are cheap, board rows are not).
The scene (< 40 KB) is built on every rank from the same descriptor, so the only data-path collective is
the exchange of finished rows, over RCCL (torch.distributed "nccl" backend = RCCL over xGMI):

* frame streams (weak scaling, the bench default): each step renders N frames, one per rank as its
  display; every frame is banded over all N ranks, each rank renders its bands of all N frames in ONE
  launch (rt_rows.frames = N, frame-major), and one all-to-all sends frame f's rows to rank f, which puts
  them in image order with rt_unshuffle_dev.  Link traffic is balanced: every rank sends and receives
  (N-1)/N of one frame per step.
* one frame split N ways (strong scaling, the c4 design): bands of a single frame, gathered to rank 0.

The reference has no distribution at all (single thread).
"""
from __future__ import annotations

from typing import List, Optional

import torch
import torch.distributed as dist

from . import abi, scenes


def auto_band_height(height: int, world: int, preferred: int = 8, equal_rows: bool = False) -> int:
    """The render's tile height, 8 rows (rt_band_plan's choice: tile-aligned bands keep the per-wave cone culling;
    ranks differ by at most one band); with `equal_rows` (frame streams: the all-to-all needs every rank's rows equal)
    the largest band height <= 16 that gives every rank the same number of rows per frame, falling back to
    `preferred` (e.g. 15 rows for 1080 rows over 8 ranks)."""
    if not equal_rows:
        return 8
    for hb in range(16, 0, -1):
        if height % (hb * world) == 0:
            return hb
    return preferred


class BandPlan:
    """Row-band partition of `frames` stacked height-row frames over `world` ranks.  equal_rows (default: frames > 1,
    the frame streams' all-to-all) asks the automatic band height for the same rows on every rank."""

    def __init__(self, height: int, world: int, band_height: Optional[int] = None, frames: int = 1,
                 equal_rows: Optional[bool] = None):
        self.height = height
        self.world = world
        self.frames = frames
        eq = frames > 1 if equal_rows is None else equal_rows
        self.band_height = band_height or auto_band_height(height, world, equal_rows=eq)
        self.frame_local = [scenes.local_rows(height, self.rows(r, 1)) for r in range(world)]
        self.local = [n * frames for n in self.frame_local]
        self.slab_rows = max(self.frame_local) if world > 0 else 0     # rows per frame, padded
        self.balanced = len(set(self.frame_local)) == 1

    def rows(self, rank: int, frames: Optional[int] = None) -> abi.rt_rows:
        return scenes.rows(self.band_height, self.world, rank, self.frames if frames is None else frames)


def _host_staged(group=None) -> bool:
    """gloo over device tensors: the rehearsal of the RCCL path on one GPU (bench.py --backend gloo) stages
    the exchange through host memory; RCCL moves device memory directly."""
    return dist.get_backend(group) == "gloo"


def gather_slabs(slab: torch.Tensor, world: int, root: int = 0, group=None) -> Optional[List[torch.Tensor]]:
    """Gather every rank's padded slab to `root` (one collective).  Returns the list on root, None elsewhere."""
    if world == 1:
        return [slab]
    rank = dist.get_rank(group)
    if slab.is_cuda and _host_staged(group):
        h = slab.cpu()
        hb = [torch.empty_like(h) for _ in range(world)] if rank == root else None
        dist.gather(h, gather_list=hb, dst=root, group=group)
        return [b.to(slab.device) for b in hb] if rank == root else None
    bufs = [torch.empty_like(slab) for _ in range(world)] if rank == root else None
    dist.gather(slab, gather_list=bufs, dst=root, group=group)
    return bufs


def exchange_frames(local: torch.Tensor, recv: torch.Tensor, world: int, async_op: bool = False, group=None):
    """Frame streams: `local` = [world frames, rows, ...] of this rank's bands (frame-major, equal rows per
    frame); after the all-to-all `recv` = [world ranks, rows, ...] holds every rank's bands of the frame this
    rank displays."""
    if world == 1:
        recv.copy_(local)
        return None
    if local.is_cuda and _host_staged(group):
        h = torch.empty(recv.shape, dtype=recv.dtype)
        dist.all_to_all_single(h, local.cpu(), group=group)
        recv.copy_(h)
        return None
    return dist.all_to_all_single(recv, local, group=group, async_op=async_op)


def assemble_on_device(slabs: torch.Tensor, plan: BandPlan, width: int, out: torch.Tensor, stream=None):
    """[world, slab_rows, W, C] (one frame's bands from every rank) -> [H, W, C] (rt_unshuffle_dev)."""
    from .tracer import unshuffle
    return unshuffle(slabs, out, width, plan.height, plan.band_height, plan.world, plan.slab_rows, stream)


def assemble_on_host(slabs, plan: BandPlan):
    """One frame from every rank's bands, on the host through the C ABI's row map (rt_global_row): used
    where no GPU is present (gloo rehearsal) and to cross-check rt_unshuffle_dev."""
    import ctypes
    import numpy as np
    L = abi.lib()
    first = np.asarray(slabs[0])
    out = np.zeros((plan.height,) + first.shape[1:], first.dtype)
    g = ctypes.c_int()
    for r in range(plan.world):
        rr = plan.rows(r, 1)
        s = np.asarray(slabs[r])
        for lr in range(plan.frame_local[r]):
            abi.check(L.rt_global_row(plan.height, ctypes.byref(rr), lr, ctypes.byref(g)), "rt_global_row")
            out[g.value] = s[lr]
    return out
