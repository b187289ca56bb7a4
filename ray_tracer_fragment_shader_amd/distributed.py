"""Image-space data parallelism across the GPUs of one node.

One process per GPU.  The frame's rows are cut into bands of `band_height` rows, dealt round-robin to the
ranks (rt_rows; contiguous stripes would be badly imbalanced: sky rows are cheap, board rows are not).
Each rank renders its bands into a dense local slab; the slabs are gathered to the display rank over
RCCL (torch.distributed "nccl" backend = RCCL over xGMI) and put back into image order there by
rt_unshuffle_dev.  The scene (< 40 KB) is built on every rank from the same descriptor, so the only
collective on the data path is the gather.  The reference has no distribution at all (single thread).
"""
from __future__ import annotations

from typing import List, Optional

import torch
import torch.distributed as dist

from . import abi, scenes


class BandPlan:
    """Row-band partition of a height-row image over `world` ranks."""

    def __init__(self, height: int, world: int, band_height: int = 8):
        self.height = height
        self.world = world
        self.band_height = band_height
        self.local = [scenes.local_rows(height, self.rows(r)) for r in range(world)]
        self.slab_rows = max(self.local) if world > 0 else 0

    def rows(self, rank: int) -> abi.rt_rows:
        return scenes.rows(self.band_height, self.world, rank)


def gather_slabs(slab: torch.Tensor, world: int, root: int = 0, group=None) -> Optional[List[torch.Tensor]]:
    """Gather every rank's padded slab to `root` (one collective).  Returns the list on root, None elsewhere."""
    if world == 1:
        return [slab]
    rank = dist.get_rank(group)
    bufs = [torch.empty_like(slab) for _ in range(world)] if rank == root else None
    dist.gather(slab, gather_list=bufs, dst=root, group=group)
    return bufs


def assemble_on_device(slabs: torch.Tensor, plan: BandPlan, width: int, out: torch.Tensor, stream=None):
    """[world, slab_rows, W, C] -> [H, W, C] in image order, on the GPU (rt_unshuffle_dev)."""
    from .tracer import unshuffle
    return unshuffle(slabs, out, width, plan.height, plan.band_height, plan.world, plan.slab_rows, stream)


def assemble_on_host(slabs, plan: BandPlan):
    """Host-side assembly through the C ABI's row map (rt_global_row): used where no GPU is present
    (gloo rehearsal) and to cross-check rt_unshuffle_dev."""
    import ctypes
    import numpy as np
    L = abi.lib()
    first = np.asarray(slabs[0])
    out = np.zeros((plan.height,) + first.shape[1:], first.dtype)
    g = ctypes.c_int()
    for r in range(plan.world):
        rr = plan.rows(r)
        s = np.asarray(slabs[r])
        for lr in range(plan.local[r]):
            abi.check(L.rt_global_row(plan.height, ctypes.byref(rr), lr, ctypes.byref(g)), "rt_global_row")
            out[g.value] = s[lr]
    return out
