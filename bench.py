#!/usr/bin/env python3
"""bench.py — Mray/s and ms/frame of the MI355X ray tracer on BASELINE.json's workload.

Workload (N=1): configs[1] of BASELINE.json = c2: 1920x1080, 8 spheres + checkerboard, 1 light,
1 reflection bounce (SURVEY.md Appendix B scene, canonical framing pitch = 500/W).  One step = one full
frame traced by rt_render_kernel (one launch) writing the RGBA32F framebuffer (unclamped HDR, the
parity image) and the RGBA8 display image, all buffers resident in HBM.  Rays are the reference's
actually-traced count (primary + reflected + shadow), taken from the kernel's own
per-pixel ray counters before the timed region and checked against the reference's pinned total.

N>1 (torch.distributed.run, one rank per GPU): `--scaling weak` (default) — frames are independent units,
so every rank renders whole frames of its own (one per step) with no data-path collective; the job's rays
per step are N frames' worth.  `--scaling streams` — N frames per step, each row-banded over all N ranks
(round-robin bands, equal rows per rank), each rank renders its bands of all N frames in ONE launch
(rt_rows.frames = N), one RCCL all-to-all sends frame f's rows to rank f, which puts them in image order
with rt_unshuffle_dev; the exchange and the assembly of step s overlap the render of step s+1
(double-buffered RGBA8 slabs, a side stream).  `--scaling strong` — ONE frame per step split over the N
ranks by row bands and gathered to rank 0 over RCCL (north_star's row-partitioned c4 design).

Printed: ONE JSON line on rank 0 (contract in the task statement) with `roofline` (HBM-write roofline of
the dominant kernel, per north_star) and `roofline_fp64` (its FP64 VALU roofline) and `cpu_baseline`
(the bit-exact C restatement, oracle/rt_oracle.c, timed on this host's cores, rank 0 at N=1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Mray/s (primary+shadow+reflect) and ms/frame at 1920×1080"
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec peak (MI355X_MICROARCH.md: 8.0 TB/s spec)
FP64_PEAK_TFLOPS = 78.6        # MI355X FP64 vector spec (an FMA counts 2)
# Algorithmic FP64 operations per frame (add, mul, div, sqrt = 1 each; SURVEY.md §8d counting restatement)
FP64_FLOPS_PER_FRAME = {"c1": 71.4e6, "c2": 1.038e9, "c3": 5.417e9, "c4": 5.417e9, "c5": 122.6e9}
BYTES_PER_PIXEL = 16 + 4       # RGBA32F framebuffer + RGBA8 display image written per pixel


def parse():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="c2", choices=["c1", "c2", "c3", "c5"])
    ap.add_argument("--scaling", default="weak", choices=["weak", "streams", "strong"])
    ap.add_argument("--band-height", type=int, default=0, help="0: auto (equal rows per rank)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-reps", type=int, default=3, help="minimum frames of the CPU baseline sample")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline sample length (wall seconds)")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="gloo: rehearse the N>1 path on a one-GPU box (every rank on device 0, exchange staged "
                         "through host memory); the measured path is nccl (= RCCL)")
    ap.add_argument("--profile-kernel-only", action="store_true",
                    help="skip parity/ray-count/cpu legs (for rocprofv3 runs)")
    return ap.parse_args()


def cpu_threads() -> int:
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        return int(env)
    try:
        return max(1, min(16, len(os.sched_getaffinity(0))))
    except AttributeError:
        return max(1, min(16, os.cpu_count() or 1))


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def main() -> int:
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    import numpy as np
    import torch
    import torch.distributed as dist

    from ray_tracer_fragment_shader_amd import scenes
    from ray_tracer_fragment_shader_amd.distributed import (BandPlan, assemble_on_device, exchange_frames,
                                                            gather_slabs)
    from ray_tracer_fragment_shader_amd.tracer import Tracer

    if not torch.cuda.is_available():
        print("bench.py needs a HIP GPU", file=sys.stderr)
        return 2
    if args.backend == "gloo" and torch.cuda.device_count() == 1:
        local = 0                                           # rehearsal: all ranks share the one GPU
    torch.cuda.set_device(local)
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")

    def barrier():
        if world > 1:
            dist.barrier()

    cfg = scenes.CONFIGS[args.config]
    W, H, B = cfg.width, cfg.height, cfg.depth
    scene = cfg.scene()
    cam = cfg.camera()
    tr = Tracer(local)
    tr.set_scene(scene)
    dev = torch.device("cuda", local)
    stream = torch.cuda.current_stream(dev)

    streams = world > 1 and args.scaling == "streams"       # banded frames + all-to-all
    strong = world > 1 and args.scaling == "strong"         # one banded frame + gather to rank 0
    banded = streams or strong                              # else: whole frames per rank, no collective
    frames = world if streams else 1                        # frames stacked in one launch on this rank
    job_frames = 1 if strong else world                     # frames the whole job renders per step
    plan = BandPlan(H, world if banded else 1, args.band_height, frames=frames)
    if streams and not plan.balanced:
        raise SystemExit(f"frame streams need equal rows per rank: H={H}, N={world}, band {plan.band_height}")
    prank = rank if banded else 0
    rows = plan.rows(rank) if banded else None
    nl = plan.local[prank]                 # rows this rank renders per step (all its frames)
    fl = plan.frame_local[prank]           # ... per frame
    out32 = torch.empty((nl, W, 4), dtype=torch.float32, device=dev)
    # RGBA8 slabs are double-buffered only where a step's exchange reads them while the next step renders
    # (frame streams, strong gather); independent frames write one buffer.
    out8 = [torch.empty((nl, W, 4), dtype=torch.uint8, device=dev) for _ in range(2 if banded else 1)]
    out8 = out8 * (2 // len(out8))
    if streams:
        recv8 = [torch.empty((world, fl, W, 4), dtype=torch.uint8, device=dev) for _ in range(2)]
        image8 = [torch.empty((H, W, 4), dtype=torch.uint8, device=dev) for _ in range(2)]
        side = torch.cuda.Stream(dev)
        assembled = [torch.cuda.Event() for _ in range(2)]
        pending = [None, None]
    elif strong and rank == 0:
        image8 = [torch.empty((H, W, 4), dtype=torch.uint8, device=dev)]

    # ---- parity + ray count (outside the timed region) ----------------------------------------------
    parity = "skipped"
    rays_frame = scenes.PINNED_RAYS.get(args.config)
    if not args.profile_kernel_only:
        chk = tr.render(cam, W, H, B, rgba32f=False, rgb64f=True, raycount=True)
        torch.cuda.synchronize()
        rc = chk["raycount"].cpu().numpy().view(np.uint32)
        rays_frame = int((rc & 0xFFFF).sum()) + int((rc >> 16).sum())
        pinned = scenes.PINNED_RAYS.get(args.config)
        if pinned is not None and rays_frame != pinned:
            raise SystemExit(f"ray count {rays_frame} != reference {pinned}")
        g = np.load(os.path.join(ROOT, "tests", "golden", f"frames_{args.config}.npz"))
        got = chk["rgb64f"].cpu().numpy()[g["pj"], g["pi"]]
        if not np.array_equal(got, g["samples"]):
            raise SystemExit(f"parity failure: max err {np.abs(got - g['samples']).max()}")
        parity = "bit-exact on 4096 sampled pixels vs the reference's rayTraceRay (tests/golden)"
        del chk, rc

    # Pre-bound launches: the ctypes argument tuples are built once, so the timed loop only issues
    # rt_render_dev (host cost ~8 us per call; a c2 frame is ~50 us, so the GPU queue stays full).
    import ctypes
    from ray_tracer_fragment_shader_amd import abi
    fn = abi.lib().rt_render_dev
    rows_ref = ctypes.byref(rows) if rows is not None else None
    launch_args = [(tr._ctx, ctypes.byref(cam), W, H, B, rows_ref, ctypes.c_void_p(out32.data_ptr()),
                    ctypes.c_void_p(out8[b].data_ptr()), None, None, ctypes.c_void_p(stream.cuda_stream))
                   for b in range(2)]
    counter = [0]

    def step():
        b = counter[0] % 2
        counter[0] += 1
        if streams and pending[b] is not None:
            pending[b].wait()                               # the all-to-all of step s-2 has read out8[b]
        rc = fn(*launch_args[b])
        if rc:
            abi.check(rc, "rt_render_dev")
        if streams:
            stream.wait_event(assembled[b])                 # recv8[b] consumed by the assembly of step s-2
            pending[b] = exchange_frames(out8[b].view(world, fl, W, 4), recv8[b], world, async_op=True)
            with torch.cuda.stream(side):
                if pending[b] is not None:
                    pending[b].wait()
                else:                                       # host-staged rehearsal: recv8[b] filled on `stream`
                    side.wait_stream(stream)
                assemble_on_device(recv8[b], plan, W, image8[b], side)
                assembled[b].record(side)
        elif strong:
            gathered = gather_slabs(out8[b], world)
            if rank == 0:
                assemble_on_device(torch.stack(gathered), plan, W, image8[0], stream)

    # Setup (untimed, independent of --warmup): the first render of this view and output set is the
    # tile-order calibration render (rt_render_dev times its tile rows and sorts them once).
    for la in launch_args:
        abi.check(fn(*la), "rt_render_dev")
    torch.cuda.synchronize()
    for _ in range(args.warmup):
        step()
    barrier()
    torch.cuda.synchronize()
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize()                                # every stream: render, exchange, assembly
    barrier()
    elapsed = time.perf_counter() - t0
    if world == 1:
        # HIP events on the launch stream bracketing the timed region, which holds only the K launches of
        # rt_render_kernel (per-launch event pairs would serialise the queue and add ~8 us per launch).
        avg_kern_ms = ev0.elapsed_time(ev1) / args.steps
    else:
        # the timed region also holds the gather: time the kernel alone in a short post-pass
        e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        n = min(args.steps, 20)
        torch.cuda.synchronize()
        e[0].record(stream)
        for _ in range(n):
            fn(*launch_args[0])
        e[1].record(stream)
        torch.cuda.synchronize()
        avg_kern_ms = e[0].elapsed_time(e[1]) / n
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    rays_step = rays_frame * job_frames
    value = rays_step * args.steps / elapsed / 1e6
    ms_step = elapsed / args.steps * 1e3

    if rank == 0:
        bytes_launch = nl * W * BYTES_PER_PIXEL
        achieved = bytes_launch / (avg_kern_ms * 1e-3) / 1e9
        flops_launch = FP64_FLOPS_PER_FRAME[args.config] * nl / H
        tflops = flops_launch / (avg_kern_ms * 1e-3) / 1e12
        traffic = None
        pmc = os.path.join(ROOT, "profiles", f"pmc_{args.config}.json")
        if os.path.exists(pmc) and world == 1:
            with open(pmc) as f:
                traffic = json.load(f).get("hbm_bytes_per_launch")
        res = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "Mray/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 4),
            "ms_per_frame": round(ms_step / job_frames, 4),
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic: canonical scene of SURVEY.md Appendix B (deterministic, no RNG)",
            "config": {
                "workload": f"{cfg.name}: {W}x{H}, {cfg.n_spheres} spheres + checkerboard, {cfg.n_lights} light(s), "
                            f"{B} bounce(s), pitch 500/W; step = {job_frames} frame(s)",
                "width": W, "height": H, "spheres": cfg.n_spheres, "lights": cfg.n_lights, "bounces": B,
                "rays_per_frame": rays_frame, "frames_per_step": job_frames,
                "parallelism": (f"frame streams: {world} frames/step, row bands (h={plan.band_height}) x {world} "
                                f"ranks, RCCL all-to-all" if streams else
                                f"row bands (h={plan.band_height}) x {world} ranks + RCCL gather to rank 0"
                                if strong else
                                f"{world} ranks x whole frames (independent frames, no collective)"
                                if world > 1 else "single GPU"),
            },
            "roofline": {
                "bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                "kernel": "rt_render_kernel", "kernel_ms": round(avg_kern_ms, 5),
                "algorithmic_bytes_per_launch": bytes_launch,
            },
            "roofline_fp64": {
                "bound": "fp64-valu", "achieved": round(tflops, 3), "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": round(tflops / FP64_PEAK_TFLOPS, 4), "flops_per_launch": flops_launch,
            },
            "parity": parity,
        }
        if world == 1 and not args.no_cpu_baseline and not args.profile_kernel_only:
            from oracle import pyoracle as po
            nt = cpu_threads()
            sa = scene.to_abi()
            # bounded sample: whole frames, repeated until --cpu-seconds of wall time (at least --cpu-reps)
            po.render(sa, cam, W, H, B, nthreads=nt)                 # warm (library load, page faults)
            frames, t0c = 0, time.perf_counter()
            while frames < args.cpu_reps or time.perf_counter() - t0c < args.cpu_seconds:
                po.render(sa, cam, W, H, B, nthreads=nt)
                frames += 1
            spent = time.perf_counter() - t0c
            res["cpu_baseline"] = {
                "value": round(rays_frame * frames / spent / 1e6, 3), "unit": "Mray/s", "cores": nt, "kind": "port",
                "sample": f"{frames} full {cfg.name} frames ({W}x{H}, {rays_frame} rays each) back to back in "
                          f"{spent:.1f} s with oracle/rt_oracle.c (bit-exact restatement, gcc -O2, OpenMP {nt} "
                          f"threads); {spent / frames * 1e3:.1f} ms/frame; host CPU: {cpu_model()}",
            }
        print(json.dumps(res), flush=True)
    tr.close()
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
