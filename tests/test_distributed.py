"""Multi-rank path on the CPU: world_size 2 (and 3) over gloo, 127.0.0.1.

Each rank renders its round-robin row bands (rt_rows) — here with the CPU oracle, since this container has
no GPU — into a padded slab; the slabs go to rank 0 with the same gather_slabs() the GPU bench uses
(RCCL there, gloo here) and rank 0 puts the rows back with the C ABI's row map (rt_global_row).  The
assembled frame must equal the single-process frame bit for bit.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, W, H, band, out_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import pyoracle as po
        from ray_tracer_fragment_shader_amd import scenes
        from ray_tracer_fragment_shader_amd.distributed import BandPlan, assemble_on_host, gather_slabs

        cfg = scenes.CONFIGS["c2"]
        plan = BandPlan(H, world, band)
        rgb, _ = po.render(cfg.scene().to_abi(), cfg.camera(W, H), W, H, cfg.depth, rows=plan.rows(rank),
                           nthreads=1)
        slab = torch.zeros((plan.slab_rows, W, 3), dtype=torch.float64)
        slab[: rgb.shape[0]] = torch.from_numpy(rgb)
        got = gather_slabs(slab, world)
        if rank == 0:
            img = assemble_on_host([g.numpy() for g in got], plan)
            np.save(out_path, img)
        else:
            assert got is None
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,band", [(2, 8), (3, 5)])
def test_row_band_gather_matches_single_process(tmp_path, world, band):
    from oracle import pyoracle as po
    from ray_tracer_fragment_shader_amd import scenes

    W, H = 96, 61
    out = str(tmp_path / "img.npy")
    mp.spawn(_worker, args=(world, _free_port(), W, H, band, out), nprocs=world, join=True)
    cfg = scenes.CONFIGS["c2"]
    want, _ = po.render(cfg.scene().to_abi(), cfg.camera(W, H), W, H, cfg.depth)
    assert np.array_equal(np.load(out), want)


def test_band_plan_balances_rows():
    from ray_tracer_fragment_shader_amd.distributed import BandPlan
    for H, G, hb in [(1080, 8, 8), (2160, 8, 8), (4320, 8, 16), (1080, 3, 8)]:
        p = BandPlan(H, G, hb)
        assert sum(p.local) == H
        assert max(p.local) - min(p.local) <= hb
        assert p.slab_rows == max(p.local)


def _stream_worker(rank, world, port, W, H, out_prefix):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import pyoracle as po
        from ray_tracer_fragment_shader_amd import scenes
        from ray_tracer_fragment_shader_amd.distributed import BandPlan, assemble_on_host, exchange_frames

        cfg = scenes.CONFIGS["c2"]
        plan = BandPlan(H, world, frames=world)
        assert plan.balanced
        rgb, _ = po.render(cfg.scene().to_abi(), cfg.camera(W, H), W, H, cfg.depth, rows=plan.rows(rank),
                           nthreads=1)
        fl = plan.frame_local[rank]
        assert rgb.shape[0] == world * fl                  # frame-major: this rank's bands of every frame
        local = torch.from_numpy(rgb).reshape(world, fl, W, 3).contiguous()
        recv = torch.empty_like(local)
        exchange_frames(local, recv, world)
        img = assemble_on_host([recv[q].numpy() for q in range(world)], plan)
        np.save(f"{out_prefix}_{rank}.npy", img)
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_frame_streams_all_to_all(tmp_path, world):
    """Weak-scaling bench layout: every rank ends up with a complete frame assembled from all ranks' bands."""
    from oracle import pyoracle as po
    from ray_tracer_fragment_shader_amd import scenes

    W, H = 80, 72
    prefix = str(tmp_path / "frame")
    mp.spawn(_stream_worker, args=(world, _free_port(), W, H, prefix), nprocs=world, join=True)
    cfg = scenes.CONFIGS["c2"]
    want, _ = po.render(cfg.scene().to_abi(), cfg.camera(W, H), W, H, cfg.depth)
    for r in range(world):
        assert np.array_equal(np.load(f"{prefix}_{r}.npy"), want)


def test_auto_band_height_balances_bench_sizes():
    from ray_tracer_fragment_shader_amd.distributed import BandPlan, auto_band_height
    for H in (480, 1080, 2160, 4320):
        for N in (1, 2, 4, 8):
            p = BandPlan(H, N, frames=N)
            assert p.balanced, (H, N, p.band_height)
            assert sum(p.frame_local) == H and p.local[0] == N * p.frame_local[0]
    assert 1080 % (auto_band_height(1080, 8) * 8) == 0
