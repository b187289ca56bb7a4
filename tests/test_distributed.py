"""Multi-rank path on the CPU: world_size 2 (and 3) over gloo, 127.0.0.1.

Each rank renders its round-robin row bands (rt_rows) — here with the CPU oracle, since this container has
no GPU — into a padded slab; the slabs go to rank 0 with the same gather_slabs() the GPU bench uses
(RCCL there, gloo here) and rank 0 puts the rows back with the C ABI's row map (rt_global_row).  The
assembled frame must equal the single-process frame bit for bit.
"""
import ctypes
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
    assert 1080 % (auto_band_height(1080, 8, equal_rows=True) * 8) == 0
    assert auto_band_height(1080, 8) == 8                     # single frames: the tile height


# ---- the product's group protocol (rt_group_plan.cpp), driven from real processes without a GPU -------------------
# rt_render_multi's host decisions — what each rank sends, where rank 0's receives land, and the scene agreement —
# are the C ABI functions below; here two (or three) gloo processes run them on their own scenes, exchange the votes
# and the real packed slabs with exactly the byte counts the plan gives, and rank 0 assembles the frame.

def _u64(words):
    return (ctypes.c_uint64 * 4)(*[int(w) for w in words])


def _pack_wire(rgb, fmt):
    """The wire image of an oracle slab (rows x W x 3 f64), as the render kernel's packed stores write it."""
    if fmt == 4:                                                   # GRAY8: the R byte of RGBA8
        return np.floor(np.clip(rgb[..., 0], 0.0, 1.0) * 255.0 + 0.5).astype(np.uint8)
    if fmt == 3:                                                   # RGB8
        return np.floor(np.clip(rgb, 0.0, 1.0) * 255.0 + 0.5).astype(np.uint8)
    if fmt == 1:                                                   # GRAY32F
        return rgb[..., 0].astype(np.float32)
    if fmt == 0:                                                   # RGBA32F
        out = np.ones(rgb.shape[:-1] + (4,), np.float32)
        out[..., :3] = rgb.astype(np.float32)
        return out
    raise AssertionError(fmt)


def _protocol_worker(rank, world, port, W, H, scene_names, outputs, out_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import pyoracle as po
        from ray_tracer_fragment_shader_amd import abi, scenes

        L = abi.lib()
        cfg = scenes.CONFIGS[scene_names[rank]] if scene_names[rank] in scenes.CONFIGS else None
        scene = cfg.scene() if cfg else _chromatic_scene()
        s_abi = scene.to_abi()
        fp, achro = ctypes.c_uint64(), ctypes.c_int()
        abi.check(L.rt_scene_fingerprint(ctypes.byref(s_abi), ctypes.byref(fp)), "rt_scene_fingerprint")
        abi.check(L.rt_scene_achromatic(ctypes.byref(s_abi), ctypes.byref(achro)), "rt_scene_achromatic")
        # --- the agreement: every rank votes before its first frame; the votes combine as ncclMax would
        assert L.rt_group_agree_due(fp.value, 0, 0) == 1
        vote = (ctypes.c_uint64 * 4)()
        L.rt_group_agree_vote(fp.value, achro.value, vote)
        mine = torch.from_numpy(np.array(list(vote), np.uint64).view(np.int64).copy())
        votes = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(votes, mine)
        acc = _u64(votes[0].numpy().view(np.uint64))
        for v in votes[1:]:
            L.rt_group_agree_combine(acc, _u64(v.numpy().view(np.uint64)))
        verdict = L.rt_group_agree_verdict(acc)
        result = {"verdict": verdict, "fp": fp.value}
        if verdict != abi.RT_OK:
            np.save(f"{out_path}_{rank}.npy", np.array([verdict], np.int64))
            dist.barrier()
            return
        # once agreed, the same scene is not voted on again — also after an X -> Y -> X round trip on one rank
        assert L.rt_group_agree_due(fp.value, 1, fp.value) == 0
        assert L.rt_group_agree_due(fp.value ^ 1, 1, fp.value) == 1
        # --- the frame plan: this rank's slab, sends, and (rank 0) receive table
        plan = abi.rt_group_plan()
        abi.check(L.rt_group_plan_frame(W, H, world, rank, 0, outputs, achro.value, ctypes.byref(plan)),
                  "rt_group_plan_frame")
        sends = torch.tensor([int(plan.send_bytes[0]), int(plan.send_bytes[1])], dtype=torch.int64)
        all_sends = [torch.empty_like(sends) for _ in range(world)]
        dist.all_gather(all_sends, sends)
        rr = rank if plan.root_renders else rank - 1          # this rank's renderer index (-1: rank 0 only assembles)
        if rr >= 0:
            rows = abi.rt_rows(plan.band_height, plan.renderers, rr, 1)
            rgb, _ = po.render(s_abi, cfg.camera(W, H) if cfg else scenes.CONFIGS["c2"].camera(W, H), W, H,
                               cfg.depth if cfg else 1, rows=rows, nthreads=1)
        else:
            rgb = np.zeros((0, W, 3))
        assert rgb.shape[0] == plan.rank_rows
        kinds = [k for k in range(2) if plan.wire[k] >= 0]
        if rank == 0:
            assert plan.send_bytes[0] == plan.send_bytes[1] == 0      # rank 0's slab is unpacked in place
            gathered = {k: np.zeros(int(plan.gather_bytes[k]), np.uint8) for k in kinds}
            total = 0
            for q in range(1, world):
                for k in kinds:
                    off, nb = ctypes.c_uint64(), ctypes.c_uint64()
                    abi.check(L.rt_group_plan_recv(ctypes.byref(plan), W, H, q, k, ctypes.byref(off),
                                                   ctypes.byref(nb)), "rt_group_plan_recv")
                    # both sides of every send / recv carry the same byte count
                    assert nb.value == int(all_sends[q][k]), (q, k, nb.value, int(all_sends[q][k]))
                    slot_bytes = plan.slab_rows * W * plan.elem_bytes[k]
                    assert off.value + nb.value <= plan.gather_bytes[k]
                    assert off.value == slot_bytes * (q if plan.root_renders else q - 1)
                    buf = torch.empty(nb.value, dtype=torch.uint8)
                    dist.recv(buf, src=q)
                    gathered[k][off.value: off.value + nb.value] = buf.numpy()
                    total += nb.value
            assert total == plan.payload_bytes
            # rank 0's own rows from its slab; peers' from their slots; image rows by the C ABI's row map
            img = {}
            for k in kinds:
                eb = plan.elem_bytes[k]
                slot = gathered[k].reshape(plan.renderers, plan.slab_rows * W * eb)
                if plan.root_renders:
                    own = np.ascontiguousarray(_pack_wire(rgb, plan.wire[k])).view(np.uint8).reshape(-1)
                    slot[0, : own.size] = own
                out = np.zeros((H, W * eb), np.uint8)
                for q in range(plan.renderers):
                    rq = abi.rt_rows(plan.band_height, plan.renderers, q, 1)
                    nl = ctypes.c_int()
                    abi.check(L.rt_local_rows(H, ctypes.byref(rq), ctypes.byref(nl)), "rt_local_rows")
                    for lr in range(nl.value):
                        j = ctypes.c_int()
                        abi.check(L.rt_global_row(H, ctypes.byref(rq), lr, ctypes.byref(j)), "rt_global_row")
                        out[j.value] = slot[q, lr * W * eb: (lr + 1) * W * eb]
                img[k] = out
            np.savez(f"{out_path}_0.npz", **{f"k{k}": img[k] for k in kinds},
                     wire=np.array([plan.wire[0], plan.wire[1]]), payload=np.array([plan.payload_bytes]))
        else:
            for k in kinds:
                data = np.ascontiguousarray(_pack_wire(rgb, plan.wire[k])).view(np.uint8).reshape(-1)
                assert data.size == plan.send_bytes[k] and plan.slab_bytes[k] >= data.size
                dist.send(torch.from_numpy(data.copy()), dst=0)
        dist.barrier()
    finally:
        dist.destroy_process_group()


def _chromatic_scene():
    """The c2 scene with a reddish light: R != G, so the wire formats are RGB8 / RGBA32F."""
    from ray_tracer_fragment_shader_amd import scenes
    sc = scenes.CONFIGS["c2"].scene()
    sc.lights[0].color = (1.0, 0.5, 0.25)
    return sc


@pytest.mark.parametrize("world,names,outputs", [
    (2, ("c2", "c2"), 3),            # achromatic: GRAY32F + GRAY8
    (3, ("chroma",) * 3, 2),         # chromatic, RGBA8 only: RGB8
    (4, ("c2",) * 4, 2),             # rank 0 only assembles: the bands go to ranks 1 .. 3
])
def test_group_protocol_plan_and_gather(tmp_path, world, names, outputs):
    from oracle import pyoracle as po
    from ray_tracer_fragment_shader_amd import abi, scenes

    W, H = 72, 50
    prefix = str(tmp_path / "proto")
    mp.spawn(_protocol_worker, args=(world, _free_port(), W, H, names, outputs, prefix), nprocs=world, join=True)
    got = np.load(f"{prefix}_0.npz")
    cfg = scenes.CONFIGS["c2"]
    scene = cfg.scene() if names[0] in scenes.CONFIGS else _chromatic_scene()
    want, _ = po.render(scene.to_abi(), cfg.camera(W, H), W, H, cfg.depth)
    for k in range(2):
        if f"k{k}" not in got:
            assert not outputs & (1 << k)
            continue
        fmt = int(got["wire"][k])
        assert fmt == ({0: abi.RT_PIXEL_GRAY32F, 1: abi.RT_PIXEL_GRAY8} if names[0] == "c2"
                       else {0: abi.RT_PIXEL_RGBA32F, 1: abi.RT_PIXEL_RGB8})[k]
        ref = np.ascontiguousarray(_pack_wire(want, fmt)).view(np.uint8).reshape(H, -1)
        assert np.array_equal(got[f"k{k}"], ref)


def test_group_protocol_scene_mismatch_fails_on_every_rank(tmp_path):
    """Ranks holding different scenes: the combined votes fail the verdict with RT_EINVAL on every rank (before
    any slab is sent), instead of mismatched send / receive sizes."""
    from ray_tracer_fragment_shader_amd import abi
    prefix = str(tmp_path / "mismatch")
    mp.spawn(_protocol_worker, args=(2, _free_port(), 40, 30, ("c2", "c3"), 3, prefix), nprocs=2, join=True)
    for r in range(2):
        assert int(np.load(f"{prefix}_{r}.npy")[0]) == abi.RT_EINVAL


@pytest.mark.parametrize("root_env", [None, "0", "1"])
def test_group_plan_matches_band_plan(monkeypatch, root_env):
    """rt_group_plan_frame against the band plan and pixel sizes it is built from, for the bench sizes: rank 0 renders
    bands below 4 ranks and only assembles from 4 on (rt_group_root_renders; RT_GROUP_ROOT_RENDERS forces either), the
    bands then going to ranks 1 .. n - 1."""
    from ray_tracer_fragment_shader_amd import abi
    if root_env is None:
        monkeypatch.delenv("RT_GROUP_ROOT_RENDERS", raising=False)
    else:
        monkeypatch.setenv("RT_GROUP_ROOT_RENDERS", root_env)
    L = abi.lib()
    for n in (1, 2, 3, 4, 8):
        want = 1 if n == 1 else (int(root_env) if root_env is not None else int(n < 4))
        assert (L.rt_group_root_renders(n) if n > 1 else 1) == want
    for W, H in ((1920, 1080), (3840, 2160), (7680, 4320), (97, 61)):
        for n in (1, 2, 3, 4, 8):
            for achro in (0, 1):
                plans = []
                for r in range(n):
                    p = abi.rt_group_plan()
                    abi.check(L.rt_group_plan_frame(W, H, n, r, 0, 3, achro, ctypes.byref(p)), "plan")
                    plans.append(p)
                root = plans[0].root_renders
                assert root == (1 if n == 1 else L.rt_group_root_renders(n))
                assert all(p.renderers == (n if root else n - 1) and p.root_renders == root for p in plans)
                hb, slab = ctypes.c_int(), ctypes.c_int()
                abi.check(L.rt_band_plan(H, plans[0].renderers, 0, ctypes.byref(hb), ctypes.byref(slab)), "rt_band_plan")
                assert all(p.band_height == hb.value and p.slab_rows == slab.value for p in plans)
                assert sum(p.rank_rows for p in plans) == H
                if not root:
                    assert plans[0].rank_rows == 0
                eb = (4, 1) if achro else (16, 3)
                for k in range(2):
                    renders = [p for p in plans if p.rank != 0 or root]
                    assert all(p.elem_bytes[k] == eb[k] and p.slab_bytes[k] == slab.value * W * eb[k] for p in renders)
                    assert root or plans[0].slab_bytes[k] == 0
                    assert sum(p.send_bytes[k] for p in plans) == (H - plans[0].rank_rows) * W * eb[k] * (n > 1)
                assert plans[0].payload_bytes == sum(p.send_bytes[0] + p.send_bytes[1] for p in plans[1:])
                if n > 1:
                    assert plans[0].gather_bytes[1] == plans[0].renderers * slab.value * W * eb[1]
                    # the receive table tiles the gather buffer: one renderer slot per peer, in renderer order
                    for q in range(1, n):
                        off, nb = ctypes.c_uint64(), ctypes.c_uint64()
                        abi.check(L.rt_group_plan_recv(ctypes.byref(plans[0]), W, H, q, 1, ctypes.byref(off),
                                                       ctypes.byref(nb)), "recv")
                        assert off.value == (q if root else q - 1) * slab.value * W * eb[1]
                        assert nb.value == plans[q].send_bytes[1]
    # misuse: a receive table asked of a rank other than 0, or of a peer out of range
    p = abi.rt_group_plan()
    abi.check(L.rt_group_plan_frame(64, 64, 2, 1, 0, 3, 1, ctypes.byref(p)), "plan")
    off, nb = ctypes.c_uint64(), ctypes.c_uint64()
    assert L.rt_group_plan_recv(ctypes.byref(p), 64, 64, 1, 0, ctypes.byref(off), ctypes.byref(nb)) == abi.RT_EINVAL
