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
per step are N frames' worth.  `--scaling strong` — ONE frame per step split over the N ranks by row bands
and gathered to rank 0 over RCCL by the C ABI's group (rt_group_create_rank + rt_render_multi: ncclSend /
ncclRecv, double-buffered slabs), north_star's row-partitioned c4 design.  `--scaling streams` — N frames
per step, each banded over all ranks, one RCCL all-to-all hands frame f to rank f (Python/torch exchange).

Extra legs in the same JSON line (outside the timed region of `value`):
  * "c4" (every N, unless --no-c4): c3's 3840x2160 frame split over the N ranks + RCCL gather to rank 0
    through rt_render_multi (N = 1: a one-rank group, ncclSend/ncclRecv to self), frames/s and Mray/s, with
    the gathered frame checked byte for byte against a one-launch render;
  * "configs" (N = 1): c3 and c5 on one GPU (ms/frame, Mray/s, HBM-write and FP64 roofline fractions);
  * "drop_in" (N = 1): rt_render, the synchronous host-buffer call that replaces draw()'s rayTraceScreen,
    per call host to host at c2 (RGBA8 back to the host), and a moving camera (a new eye every frame);
  * "roofline" / "roofline_fp64" of the dominant kernel and "cpu_baseline" (the reference's own rayTraceRay built
    from its sources, oracle/_ref, when the build travelled with the tree, else the bit-exact C restatement
    oracle/rt_oracle.c; best of 3 blocks of whole frames on this host's CPU share, rank 0 at N=1 only).
"""
from __future__ import annotations

import argparse
import ctypes
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


def parse(argv=None):
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
                    help="skip parity/ray-count/cpu and extra legs (for rocprofv3 runs)")
    ap.add_argument("--no-c4", action="store_true", help="skip the c4 (row split + RCCL gather) leg")
    ap.add_argument("--c4-timeout", type=float, default=240.0,
                    help="seconds the c4 leg may take before the job prints its line without it and exits")
    ap.add_argument("--no-extra", action="store_true", help="skip the c3/c5 and drop-in legs (N = 1)")
    ap.add_argument("--frames-in-flight", type=int, default=3,
                    help="independent frames round-robin over this many HIP streams, each with its own context and "
                         "output buffers, so a frame's launch starts while the previous frame's last waves drain "
                         "(1: one stream, launches back to back)")
    ap.add_argument("--settle", type=float, default=0.25,
                    help="seconds of untimed back-to-back frames before the warm-up steps, so the GPU clock reaches "
                         "its loaded steady state (MI355X_MICROARCH.md 'DVFS give-back')")
    ap.add_argument("--dry-launch", action="store_true",
                    help="print how this command would run (one process, or the per-rank child commands of "
                         "--gpus N without a launcher) and exit without touching the GPU")
    return ap.parse_args(argv)


# ---- launch decision ---------------------------------------------------------------------------------------------
# `--gpus N` is authoritative.  Under a launcher (torch.distributed.run sets WORLD_SIZE) the world size must equal
# N.  Without one, N > 1 makes this process a launcher itself: it starts N fresh child ranks (one process per GPU,
# the same RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* environment torch.distributed.run gives them), relays rank 0's
# JSON line and exits with the worst child exit code.  The parent never initialises HIP (device counting through
# torch.cuda.device_count() does not, on this image).

def launch_plan(args, env, argv, device_count=None):
    """("run", world) — bench in this process; ("launch", [(env, cmd), ...]) — start these child ranks;
    ("error", message) — refuse.  `device_count` (callable) is consulted only for an nccl self-launch."""
    ws = env.get("WORLD_SIZE")
    if args.gpus < 1:
        return "error", f"--gpus must be >= 1 (got {args.gpus})"
    if ws is not None:
        try:
            w = int(ws)
        except ValueError:
            return "error", f"WORLD_SIZE={ws!r} is not an integer"
        if w != args.gpus:
            return "error", (f"WORLD_SIZE={w} (from the launcher) but --gpus {args.gpus}: the job would not measure "
                             f"the GPU count it claims; launch {args.gpus} rank(s) or pass --gpus {w}")
        return "run", w
    if args.gpus == 1:
        return "run", 1
    n = args.gpus
    if args.backend == "nccl" and device_count is not None:
        have = device_count()
        if have < n:
            return "error", (f"--gpus {n} with the nccl (RCCL) backend needs {n} GPUs, this host shows {have}; "
                             f"rehearse the N>1 path on fewer GPUs with --backend gloo")
    port = env.get("MASTER_PORT") or str(free_port())
    child_argv = [a for a in argv if a != "--dry-launch"]
    ranks = []
    for r in range(n):
        e = {"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(n), "LOCAL_WORLD_SIZE": str(n),
             "GROUP_RANK": "0", "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": port}
        ranks.append((e, [sys.executable, os.path.abspath(__file__)] + child_argv))
    return "launch", ranks


def free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def run_ranks(ranks, out, grace_s=60.0) -> int:
    """Start the child ranks, relay rank 0's JSON line to `out`, return the worst exit code.  A rank that fails
    leaves the others `grace_s` seconds to finish (a peer blocked in a collective never would); then they are
    terminated (exact PIDs) and counted as failed."""
    import subprocess
    import threading

    procs = []
    for e, cmd in ranks:
        env = dict(os.environ)
        env.update(e)
        procs.append(subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE if e["RANK"] == "0" else subprocess.DEVNULL,
                                      stderr=None, text=True))
    lines = []

    def pump():
        for line in procs[0].stdout:
            s = line.strip()
            if s.startswith("{") and '"metric"' in s:
                lines.append(s)
            elif s:
                print(s, file=sys.stderr, flush=True)
    th = threading.Thread(target=pump, daemon=True)
    th.start()
    first_fail = None
    while True:
        codes = [p.poll() for p in procs]
        if all(c is not None for c in codes):
            break
        if first_fail is None and any(c not in (None, 0) for c in codes):
            first_fail = time.monotonic()
        if first_fail is not None and time.monotonic() - first_fail > grace_s:
            for p in procs:
                if p.poll() is None:
                    print(f"bench.py: terminating rank pid {p.pid} (a peer failed {grace_s:g} s ago)", file=sys.stderr)
                    p.terminate()
            for p in procs:
                try:
                    p.wait(timeout=15)
                except subprocess.TimeoutExpired:
                    p.kill()
                    p.wait()
            break
        time.sleep(0.05)
    th.join(timeout=10)
    codes = [p.returncode for p in procs]
    for r, c in enumerate(codes):
        if c:
            print(f"bench.py: rank {r} exited with {c}", file=sys.stderr)
    worst = max(codes, key=lambda c: (c != 0, abs(c))) if codes else 1
    if lines:
        print(lines[-1], file=out, flush=True)
    elif worst == 0:
        print("bench.py: rank 0 printed no JSON line", file=sys.stderr)
        worst = 1
    return 128 - worst if worst < 0 else worst         # killed by signal k: 128 + k, as a shell reports it


def affinity_cores() -> int:
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def cpu_threads() -> int:
    """Every core of the affinity mask, unless the launcher set OMP_NUM_THREADS (the GPU boxes set it to
    the box's CPU share, 16 per GPU, and their rules say to keep it)."""
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        return int(env)
    return max(1, affinity_cores())


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def kernel_rooflines(cfg_name, nl, W, H, avg_kern_ms):
    """HBM-write roofline of rt_render_kernel (north_star's figure) and its FP64 VALU roofline.

    FP64: `achieved` = FP64 flops the kernel ISSUED per launch (PMC: (ADD + MUL + TRANS + 2 FMA)_F64
    wave-instructions x 64 lanes, profiles/pmc_<cfg>.json, an upper bound since masked lanes count) / the
    measured launch time.  The reference's own op count (a brute-force walk of every sphere)
    is reported beside it as `reference_equivalent_tflops`: the kernel skips provably-missed tests, so that
    rate can exceed the FP64 peak (c5) and is not a utilisation."""
    bytes_launch = nl * W * BYTES_PER_PIXEL
    achieved = bytes_launch / (avg_kern_ms * 1e-3) / 1e9
    ref_flops = FP64_FLOPS_PER_FRAME[cfg_name] * nl / H
    traffic = issued = None
    pmc = os.path.join(ROOT, "profiles", f"pmc_{cfg_name}.json")
    if os.path.exists(pmc):
        with open(pmc) as f:
            pm = json.load(f)
        traffic = pm.get("hbm_bytes_per_launch")
        issued = pm.get("fp64_flops_issued_per_launch")
    if issued is not None:
        issued *= nl / H
    tflops = issued / (avg_kern_ms * 1e-3) / 1e12 if issued is not None else None
    return ({"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
             "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic, "kernel": "rt_render_kernel",
             "kernel_ms": round(avg_kern_ms, 5), "algorithmic_bytes_per_launch": bytes_launch},
            {"bound": "fp64-valu", "achieved": round(tflops, 3) if tflops is not None else None,
             "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
             "frac": round(tflops / FP64_PEAK_TFLOPS, 4) if tflops is not None else None,
             "flops_issued_per_launch": issued, "flops_source": f"profiles/pmc_{cfg_name}.json (PMC, issued)",
             "reference_equivalent_tflops": round(ref_flops / (avg_kern_ms * 1e-3) / 1e12, 3),
             "reference_flops_per_launch": ref_flops})


ROCPROF_ONE_STREAM = "profiles/r06/{cfg}_kernel_stats_1stream.csv"


def rocprof_reference(cfg_name, full_frame):
    """The committed one-stream rocprofv3 --kernel-trace --stats summary of this config (tools/gpu_r06.sh STEPS=prof:
    bench.py --frames-in-flight 1 --profile-kernel-only): AverageNs of rt_render_kernel is the launch duration,
    so bytes / AverageNs / peak reproduces `frac` from profiles/ alone."""
    path = os.path.join(ROOT, ROCPROF_ONE_STREAM.format(cfg=cfg_name))
    if not full_frame or not os.path.exists(path):
        return None
    import csv
    with open(path) as f:
        for row in csv.DictReader(f):
            if row.get("Name", "").startswith("void rtk::rt_render_kernel") or "rt_render_kernel" in row.get("Name", ""):
                avg_us = float(row["AverageNs"]) / 1e3
                return {"rocprof_avg_us": round(avg_us, 3), "rocprof_calls": int(row["Calls"]),
                        "rocprof_source": ROCPROF_ONE_STREAM.format(cfg=cfg_name)}
    return None


_STREAM_POOL = []


def frame_streams(torch, dev, stream, n):
    """The bench's stream and n - 1 more for frames in flight, the same streams for every leg (created together at
    start-up: HIP gives each new stream one of four hardware queues in creation order, and streams created later can
    share the bench stream's queue and serialise frames meant to overlap)."""
    while len(_STREAM_POOL) < n - 1:
        _STREAM_POOL.append(torch.cuda.Stream(dev))
    return [stream] + _STREAM_POOL[:n - 1]


def pipelined_frames(torch, L, abi, trs, sts, launch_args, steps, settle_s):
    """Untimed settle, then `steps` frames round-robin over the streams `sts` (launch_args[i] on sts[i]).
    Returns (wall seconds, per-frame interval in ms from HIP events bracketing all streams)."""
    n = len(launch_args)
    fn = L.rt_render_dev
    t_end = time.perf_counter() + settle_s
    k = 0
    while time.perf_counter() < t_end or k < 2 * n:
        for _ in range(16):
            abi.check(fn(*launch_args[k % n]), "rt_render_dev")
            k += 1
        torch.cuda.synchronize()
    s0 = sts[0]
    ev0 = torch.cuda.Event(enable_timing=True)
    ends = [torch.cuda.Event(enable_timing=True) for _ in sts]
    # The interval's events: a start stamp on the first stream and an end stamp on every stream, compared afterwards
    # (no cross-stream waits inside the timed region: they only delayed its first launch and its end).  The start
    # stamp is recorded just before the timer starts (the GPU is idle: it lands at once), so the timed region holds
    # the frames' launches, their execution and the final synchronisation only.
    ev0.record(s0)
    t0 = time.perf_counter()
    for i in range(steps):
        rc = fn(*launch_args[i % n])
        if rc:
            abi.check(rc, "rt_render_dev")
    for e, s in zip(ends, sts):
        e.record(s)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    return wall, max(ev0.elapsed_time(e) for e in ends) / steps


def serial_kernel_ms(torch, L, abi, launch, stream, n=20):
    """Average duration of `n` back-to-back launches on one stream (HIP events on that stream)."""
    e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    torch.cuda.synchronize()
    e[0].record(stream)
    for _ in range(n):
        abi.check(L.rt_render_dev(*launch), "rt_render_dev")
    e[1].record(stream)
    torch.cuda.synchronize()
    return e[0].elapsed_time(e[1]) / n


HBM_PEAK_GBS = 8000.0
SETTLE_FRAMES_PER_S = 10000                            # c4 settle: frames per second of --settle (a c3 frame is ~0.11 ms)


def settle_frames(settle_s):
    """Untimed frames a group leg runs before timing: the same count on every rank (each frame is a collective)."""
    return max(0, int(round(settle_s * SETTLE_FRAMES_PER_S)))


def c4_scaling_keys(n, W, H, rays, c4_ms, c3_ms_inflight, c3_ms_serial):
    """The c4 leg's scaling figures against the same job's one-GPU c3 frame (measured on rank 0 before the group
    leg, same scene, view and RGBA8 output): speedup = one GPU's best c3 frame time (frames in flight) / the split
    frame's time, efficiency = speedup / n; also against the one-stream serial c3 frame.  HBM-write fraction per GPU
    = the RGBA8 image's bytes (W x H x 4) shared over n GPUs per split frame, against HBM_PEAK_GBS."""
    out = {"c3_1gpu_ms_per_frame": round(c3_ms_inflight, 5), "c3_1gpu_ms_serial": round(c3_ms_serial, 5)}
    if not c4_ms or c4_ms <= 0:
        return out
    sp = c3_ms_inflight / c4_ms
    out.update({
        "speedup_vs_c3_1gpu": round(sp, 3),
        "efficiency": round(sp / n, 3),
        "speedup_vs_c3_1gpu_serial": round(c3_ms_serial / c4_ms, 3),
        "mray_s_per_gpu": round(rays / (c4_ms * 1e-3) / 1e6 / n, 3),
        "hbm_write_frac_per_gpu": round((W * H * 4 / n) / (c4_ms * 1e-3) / (HBM_PEAK_GBS * 1e9), 5),
    })
    return out


GROUP_BUFFERS = 3                                      # rt_group.cpp kBufs: frame buffers per rank
XGMI_LINK_GBS = 153.0                                   # nominal per-link rate (7 links per MI355X); not measured here


def c4_projection_keys(n, c3_ms_per_frame, rank_ms, unpack_ms, slab_bytes, root_ms=None, root_renders=True):
    """One GPU's projection of an n-rank c4 frame (rt_render_multi at n ranks cannot run on one GPU): every rank's band
    set rendered alone the way the group renders it (rank_ms[r], per frame, frames in flight as the group keeps them),
    and rank 0's unpack of the n-rank gathered buffer (unpack_ms, alone).  root_ms: rank 0's own pipeline measured as
    the group runs it — its bands on the render streams and, per frame, the unpack on its high-priority comm stream
    behind that frame's render — so the unpack overlaps the next render; without it rank 0 is charged its render plus
    the whole unpack.  Projected frame interval = the slowest stage: max(rank_ms[1:], rank 0), or the gather (each
    peer's slab_bytes over its own xGMI link into rank 0, double-buffered behind the next render) at the nominal link
    rate — not measured — when that is longer.  root_renders False (rt_group_root_renders, from 4 ranks): rank_ms are
    the n - 1 renderers' (ranks 1 .. n - 1) and rank 0 only receives and unpacks (root_ms, or unpack_ms)."""
    render = max(rank_ms)
    if root_renders:
        root = root_ms if root_ms is not None else rank_ms[0] + unpack_ms
        peers = rank_ms[1:]
    else:
        root = root_ms if root_ms is not None else unpack_ms
        peers = rank_ms
    frame = max(max(peers, default=0.0), root)
    xfer = slab_bytes / (XGMI_LINK_GBS * 1e9) * 1e3
    bound = max(frame, xfer)
    key = f"n{n}"
    out = {f"{key}_root_renders": bool(root_renders),
           f"{key}_rank_render_ms": [round(x, 5) for x in rank_ms], f"{key}_rank_render_ms_max": round(render, 5),
           f"{key}_unpack_ms": round(unpack_ms, 5), f"{key}_rank0_ms": round(root, 5),
           f"{key}_projected_frame_ms": round(bound, 5), f"{key}_gather_ms_nominal": round(xfer, 5),
           f"{key}_limiting_stage": ("gather (nominal xGMI)" if xfer > frame else
                                     ("rank 0 (bands + unpack)" if root_renders else "rank 0 (unpack)")
                                     if root >= frame else "a peer's band render"),
           f"{key}_speedup_bound": round(c3_ms_per_frame / bound, 3)}
    return out


def c4_parallelism_text(n, c4):
    """The top-level `parallelism` suffix that carries the row-split c4 curve at N > 1 (SCALE records)."""
    if not c4 or "speedup_vs_c3_1gpu" not in c4:
        return ""
    return (f"; c4 (one 3840x2160 frame row-split over {n} GPUs, RGBA8 gathered to rank 0): {c4.get('value')} Mray/s, "
            f"{c4['mray_s_per_gpu']} Mray/s per GPU, {c4['speedup_vs_c3_1gpu']}x one GPU's c3 frame "
            f"(efficiency {c4['efficiency']}), HBM-write {c4['hbm_write_frac_per_gpu']} of peak per GPU")


def c3_one_gpu(torch, L, abi, Tracer, cfg, dev, local, nfly, steps, settle_s):
    """One GPU's c3 frame as the c4 leg's denominator: RGBA8 only (the group leg's output), calibrated view, `nfly`
    frames in flight on their own streams (the bench's timed pattern) and one stream serial, after `settle_s` seconds of
    untimed frames (the GPU's clocks ramp up under load: a leg timed right after an idle stretch measured 14% slower,
    tools/c4_gap_probe.py).  -> (ms in flight, ms serial)."""
    W, H, B = cfg.width, cfg.height, cfg.depth
    cam = cfg.camera()
    ts = [Tracer(local) for _ in range(nfly)]
    for t in ts:
        t.set_scene(cfg.scene())
    ss = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(nfly - 1)]
    outs = [torch.empty((H, W, 4), dtype=torch.uint8, device=dev) for _ in range(nfly)]
    la = [(ts[i]._ctx, ctypes.byref(cam), W, H, B, None, None, ctypes.c_void_p(outs[i].data_ptr()), None, None,
           ctypes.c_void_p(ss[i].cuda_stream)) for i in range(nfly)]
    for _ in range(2):                                       # first render + the calibration render of the view
        for a in la:
            abi.check(L.rt_render_dev(*a), "rt_render_dev")
    torch.cuda.synchronize()
    _, ms_fly = pipelined_frames(torch, L, abi, ts, ss, la, steps, settle_s)
    ms_ser = serial_kernel_ms(torch, L, abi, la[0], ss[0], n=steps)
    for t in ts:
        t.close()
    return ms_fly, ms_ser


def c4_rank_projection(torch, L, abi, Tracer, cfg, dev, local, n, band_height, c3_ms_per_frame, frames=120):
    """One GPU's projection of the c4 frame at n ranks (c4_projection_keys): each rank r's band set (rt_rows(hb, n, r),
    the band plan rt_render_multi uses) rendered alone as the group renders it — GRAY8 wire format into a slab, the
    rank's two render streams taking frames in turn, one context per rank — timed over `frames` frames after the
    calibration renders; then rank 0's rt_unpack_dev of an n-rank gathered GRAY8 buffer into the RGBA8 image."""
    W, H, B = cfg.width, cfg.height, cfg.depth
    cam = cfg.camera()
    # the group's plan: from 4 ranks rank 0 only assembles and the bands go to ranks 1 .. n - 1 (rt_group_root_renders)
    plan = abi.rt_group_plan()
    abi.check(L.rt_group_plan_frame(W, H, n, 0, band_height, abi.RT_OUT_RGBA8, 1, ctypes.byref(plan)), "plan")
    hb, sr, nr, root_renders = plan.band_height, plan.slab_rows, plan.renderers, bool(plan.root_renders)
    sts = [torch.cuda.Stream(dev) for _ in range(2)]
    rank_ms = []
    for r in range(nr):                                      # renderer r (rank r, or r + 1 when rank 0 assembles)
        t = Tracer(local)
        t.set_scene(cfg.scene())
        rows = abi.rt_rows(hb, nr, r, 1)
        slabs = [torch.empty((sr, W), dtype=torch.uint8, device=dev) for _ in range(2)]
        la = [(t._ctx, ctypes.byref(cam), W, H, B, ctypes.byref(rows), abi.RT_PIXEL_GRAY32F, None, abi.RT_PIXEL_GRAY8,
               ctypes.c_void_p(slabs[k].data_ptr()), ctypes.c_void_p(sts[k].cuda_stream)) for k in range(2)]
        for _ in range(3):                                   # first render and calibration of the rank's view
            abi.check(L.rt_render_dev_packed(*la[0]), "rt_render_dev_packed")
        abi.check(L.rt_render_dev_packed(*la[1]), "rt_render_dev_packed")
        for f in range(frames // 2):                          # warm (untimed)
            abi.check(L.rt_render_dev_packed(*la[f & 1]), "rt_render_dev_packed")
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for f in range(frames):
            rc = L.rt_render_dev_packed(*la[f & 1])
            if rc:
                abi.check(rc, "rt_render_dev_packed")
        torch.cuda.synchronize()
        rank_ms.append((time.perf_counter() - t0) * 1e3 / frames)
        t.close()
    gathered = torch.zeros((nr * sr, W), dtype=torch.uint8, device=dev)
    img = torch.empty((H, W, 4), dtype=torch.uint8, device=dev)
    ua = (ctypes.c_void_p(gathered.data_ptr()), ctypes.c_void_p(img.data_ptr()), W, H, abi.RT_PIXEL_GRAY8,
          abi.RT_PIXEL_RGBA8, hb, nr, sr, ctypes.c_void_p(sts[0].cuda_stream))
    for _ in range(10):
        abi.check(L.rt_unpack_dev(*ua), "rt_unpack_dev")
    e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    torch.cuda.synchronize()
    e[0].record(sts[0])
    for _ in range(40):
        abi.check(L.rt_unpack_dev(*ua), "rt_unpack_dev")
    e[1].record(sts[0])
    torch.cuda.synchronize()
    unpack_ms = e[0].elapsed_time(e[1]) / 40
    # rank 0 as rt_render_multi runs it: bands on the two render streams in turn into three frame buffers, each frame's
    # unpack (its slab and the gathered peers' bands, pre-filled) on the comm stream (default priority, as the group)
    # behind that frame's render
    t = Tracer(local)
    t.set_scene(cfg.scene())
    rows = abi.rt_rows(hb, nr, 0, 1)
    nb = GROUP_BUFFERS
    gath = [torch.zeros((nr * sr, W), dtype=torch.uint8, device=dev) for _ in range(nb)]
    cs = torch.cuda.Stream(dev)
    ev_r = [torch.cuda.Event() for _ in range(nb)]
    ev_a = [torch.cuda.Event() for _ in range(nb)]
    la = [(t._ctx, ctypes.byref(cam), W, H, B, ctypes.byref(rows), abi.RT_PIXEL_GRAY32F, None, abi.RT_PIXEL_GRAY8,
           ctypes.c_void_p(gath[b].data_ptr())) for b in range(nb)]
    ub = [(ctypes.c_void_p(gath[b].data_ptr()), ctypes.c_void_p(img.data_ptr()), W, H, abi.RT_PIXEL_GRAY8,
           abi.RT_PIXEL_RGBA8, hb, nr, sr, ctypes.c_void_p(cs.cuda_stream)) for b in range(nb)]
    used = [False] * nb

    def root_frame(f):
        b, k = f % nb, f & 1
        if root_renders:                                      # (an assembling rank 0: the unpack alone)
            if used[b]:
                sts[k].wait_event(ev_a[b])                    # frame f - nb's unpack has read buffer b
            abi.check(L.rt_render_dev_packed(*la[b], ctypes.c_void_p(sts[k].cuda_stream)), "rt_render_dev_packed")
            ev_r[b].record(sts[k])
            cs.wait_event(ev_r[b])
        abi.check(L.rt_unpack_dev(*ub[b]), "rt_unpack_dev")
        ev_a[b].record(cs)
        used[b] = True
    for f in range(3 + frames // 2):
        root_frame(f)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for f in range(frames):
        root_frame(f)
    torch.cuda.synchronize()
    root_ms = (time.perf_counter() - t0) * 1e3 / frames
    t.close()
    keys = c4_projection_keys(n, c3_ms_per_frame, rank_ms, unpack_ms, sr * W, root_ms=root_ms, root_renders=root_renders)
    keys[f"n{n}_band_height"] = hb
    return keys


def packed_host_legs(t, sa, cam, W, H, B, k=30):
    """draw()'s host frame in the narrowest exact format (rt_render_packed, GRAY8 for the achromatic c2 scene:
    2.1 MB over PCIe instead of 8.3 MB), synchronous and pipelined (rt_render_packed_async + rt_ctx_wait: the copy of
    frame k runs beside the render of frame k+1), into pinned memory from rt_host_alloc."""
    import ctypes

    from ray_tracer_fragment_shader_amd import abi
    L = abi.lib()
    pins = []
    for _ in range(3):
        p = ctypes.c_void_p()
        abi.check(L.rt_host_alloc(W * H, ctypes.byref(p)), "rt_host_alloc")
        pins.append(p)
    out = {}
    try:
        fmt = abi.RT_PIXEL_GRAY8
        a = (t._ctx, ctypes.byref(sa), ctypes.byref(cam), W, H, B, fmt)
        for _ in range(3):
            abi.check(L.rt_render_packed(*a, pins[0], None), "rt_render_packed")
        t0 = time.perf_counter()
        for _ in range(k):
            abi.check(L.rt_render_packed(*a, pins[0], None), "rt_render_packed")
        out["rt_render_packed_gray8_ms_per_call"] = round((time.perf_counter() - t0) / k * 1e3, 4)
        tk = [ctypes.c_uint64() for _ in range(3)]
        for depth, key in ((1, "rt_render_packed_async_gray8_ms_per_frame"),
                           (2, "rt_render_packed_async_gray8_ms_per_frame_2_behind")):
            for f in range(4):
                abi.check(L.rt_render_packed_async(*a, pins[f % 3], ctypes.byref(tk[f % 3])), "rt_render_packed_async")
            abi.check(L.rt_ctx_wait(t._ctx, 0), "rt_ctx_wait")
            t0 = time.perf_counter()
            for f in range(k):                              # the draw() loop: queue frame f, show frame f - depth
                abi.check(L.rt_render_packed_async(*a, pins[f % 3], ctypes.byref(tk[f % 3])), "rt_render_packed_async")
                if f >= depth:
                    abi.check(L.rt_ctx_wait(t._ctx, tk[(f - depth) % 3].value), "rt_ctx_wait")
            abi.check(L.rt_ctx_wait(t._ctx, 0), "rt_ctx_wait")
            out[key] = round((time.perf_counter() - t0) / k * 1e3, 4)
        out["packed_note"] = ("c2 frame as GRAY8 (2.07 MB: the scene is achromatic, rt_scene_achromatic) into pinned "
                              "memory: synchronous per call (render + copy kernel on the render stream), and pipelined "
                              "(queue frame f, wait for frame f-1 — one frame of latency — or f-2: each frame's copy "
                              "runs on an SDMA engine, started by the render stream, beside the next frame's render)")
    finally:
        for p in pins:
            L.rt_host_free(p)
    return out


def dropin_binding_legs(W, H, B, cfg, frames=30):
    """INTEGRATION.md's C++ binding (lib/rt_dropin: loadScene/draw()/writePpmScreenshot) on the c2 board — light b6,
    the 8 spheres of SURVEY.md Appendix B — at 1920x1080, pitch 500/W, depth 1: its own 'ms per draw()' over
    `frames` frames, as the r02 binding ran it (pageable RGBA8) and as it runs now (pinned, auto = GRAY8; and
    pipelined)."""
    import subprocess
    import tempfile
    exe = os.path.join(ROOT, "ray_tracer_fragment_shader_amd", "lib", "rt_dropin")
    entries = ["b6:a"] + [f"{sq}:d" for sq in ("d7", "b2", "f5", "h8", "c4", "e2", "g6", "a5")]
    res = {}
    with tempfile.TemporaryDirectory() as td:
        for name, opts in (("pageable_rgba8", ["--pageable", "--format", "rgba"]), ("pinned_auto", []),
                           ("pinned_auto_pipelined", ["--pipelined"])):
            cmd = [exe, "--frames", str(frames), "--width", str(W), "--height", str(H), "--pitch", repr(500.0 / W),
                   "--depth", str(B), "--out", os.path.join(td, "f.ppm")] + opts + entries
            try:
                r = subprocess.run(cmd, capture_output=True, text=True, timeout=120)
                line = r.stdout.strip().splitlines()[-1] if r.stdout.strip() else r.stderr.strip()
                ms = float(line.split(" ms per draw()")[0].rsplit(" ", 1)[1]) if r.returncode == 0 else None
                res[name] = {"ms_per_draw": ms, "output": line}
            except Exception as exc:                        # reported, the timed metric stands
                res[name] = {"error": f"{type(exc).__name__}: {exc}"}
    res["note"] = (f"lib/rt_dropin --frames {frames} (the committed INTEGRATION.md binding, C++, built against "
                   "rt_api.h): its own steady-state ms per draw() after the first three frames (scene upload, first render, "
                   "calibration render), host to host")
    return res


def cpu_sample(render, seconds):
    """Best of 3 blocks of whole frames, each about seconds / 3 of wall time -> (blocks [(frames, s)], best)."""
    render()                                                 # warm (library load, page faults)
    blocks = []
    for _ in range(3):
        n, t0 = 0, time.perf_counter()
        while n < 1 or time.perf_counter() - t0 < seconds / 3:
            render()
            n += 1
        blocks.append((n, time.perf_counter() - t0))
    return blocks, max(blocks, key=lambda b: b[0] / b[1])


def cpu_baseline_labels(nt, env=None):
    """What the CPU sample ran on: `threads` = the OpenMP threads used — the lease's CPU share (OMP_NUM_THREADS, 16 on
    the GPU boxes), hardware threads, not physical cores; `cores` repeats it because the bench contract names that key
    (its meaning is `threads`, stated in `threads_note`); `nproc` and `affinity_threads` = the machine's hardware threads
    and those this process may run on."""
    env = os.environ if env is None else env
    return {"unit": "Mray/s", "threads": nt, "cores": nt,
            "threads_note": (f"{nt} OpenMP threads = the lease's CPU share (OMP_NUM_THREADS="
                             f"{env.get('OMP_NUM_THREADS')}) of a {os.cpu_count()}-hardware-thread host; hardware "
                             "threads, not physical cores ('cores' = the same count, the key the bench contract names)"),
            "nproc": os.cpu_count(), "affinity_threads": affinity_cores(),
            "omp_num_threads_env": env.get("OMP_NUM_THREADS"), "host_cpu": cpu_model()}


def cpu_baseline(args, cfg, scene, cam, W, H, B, rays_frame):
    """The CPU path timed on this host (rank 0, N = 1): the reference's own rayTraceRay compiled from its sources
    (oracle/_ref/libref.so: built in the build container by oracle/Makefile, it travels with the tree; kind
    "reference") when present, over the same rows with OpenMP on the host's CPU share, checked against the golden
    frame hash; else the bit-exact C restatement (kind "port").  The port is timed beside it either way."""
    from oracle import pyoracle as po
    from tests import golden
    nt = cpu_threads()
    sa = scene.to_abi()
    pblocks, pbest = cpu_sample(lambda: po.render(sa, cam, W, H, B, nthreads=nt),
                                args.cpu_seconds / 2 if os.path.exists(po.REF_SO) else args.cpu_seconds)
    port = rays_frame * pbest[0] / pbest[1] / 1e6
    n1, t1 = 0, time.perf_counter()                          # one thread, for the per-core rate
    while n1 < 1 or time.perf_counter() - t1 < 2.0:
        po.render(sa, cam, W, H, B, nthreads=1)
        n1 += 1
    per_core = rays_frame * n1 / (time.perf_counter() - t1) / 1e6
    common = cpu_baseline_labels(nt)
    port_desc = (f"oracle/rt_oracle.c (bit-exact restatement, gcc -O2 -ffp-contract=off -fopenmp, OpenMP {nt} threads, "
                 f"schedule(dynamic,1) over rows): best of 3 blocks of whole {cfg.name} frames "
                 f"({', '.join(str(b[0]) for b in pblocks)} frames in {', '.join(f'{b[1]:.1f}' for b in pblocks)} s)")
    if os.path.exists(po.REF_SO):
        try:
            rgb = po.ref_render(scene, W, H, B, cam.pitch, nthreads=nt)
            want = golden.manifest()["frames"].get(cfg.name, {}).get("fnv1a64")
            ref_hash = f"{po.fnv1a64(rgb):016x}"
            rblocks, rbest = cpu_sample(lambda: po.ref_render(scene, W, H, B, cam.pitch, nthreads=nt), args.cpu_seconds / 2)
            val = rays_frame * rbest[0] / rbest[1] / 1e6
            return {"value": round(val, 3), "kind": "reference", **common,
                    "sample": f"best of 3 blocks of whole {cfg.name} frames ({W}x{H}, {rays_frame} rays each; blocks of "
                              f"{', '.join(str(b[0]) for b in rblocks)} frames in "
                              f"{', '.join(f'{b[1]:.1f}' for b in rblocks)} s) traced by the reference's own "
                              f"rayTraceRay (Hw4/MySdlApplication.cpp:1184-1249 compiled from its sources, "
                              f"oracle/_ref/libref.so, g++ -O2), OpenMP {nt} threads over rows; "
                              f"{rbest[1] / rbest[0] * 1e3:.1f} ms/frame",
                    "reference_frame_fnv1a64": ref_hash, "reference_frame_matches_golden": ref_hash == want,
                    "port_value": round(port, 3), "port_sample": port_desc,
                    "port_one_thread_value": round(per_core, 3)}
        except Exception as exc:                             # reported; the port stands in
            common["reference_error"] = f"{type(exc).__name__}: {exc}"
    return {"value": round(port, 3), "kind": "port", **common,
            "sample": f"{port_desc}; {pbest[1] / pbest[0] * 1e3:.1f} ms/frame",
            "one_thread_value": round(per_core, 3),
            "all_affinity_cores_linear_estimate": round(per_core * affinity_cores(), 3)}


def torch_device_count() -> int:
    import torch
    return torch.cuda.device_count()                   # counts devices without initialising HIP (this image)


def main() -> int:
    argv = sys.argv[1:]
    args = parse(argv)
    kind, plan_or_msg = launch_plan(args, os.environ, argv, device_count=torch_device_count)
    if kind == "error":
        print(f"bench.py: {plan_or_msg}", file=sys.stderr)
        return 2
    if args.dry_launch:
        if kind == "run":
            print(json.dumps({"launch": "in-process", "world_size": plan_or_msg}))
        else:
            print(json.dumps({"launch": "children", "world_size": len(plan_or_msg),
                              "ranks": [{"env": e, "cmd": c} for e, c in plan_or_msg]}))
        return 0
    if kind == "launch":
        return run_ranks(plan_or_msg, sys.stdout)
    # The JSON line goes to the process's original stdout; whatever native libraries write to fd 1 (RCCL prints
    # its version banner there at communicator init) is sent to stderr, so stdout carries exactly one line.
    sys.stdout.flush()
    out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    world = plan_or_msg
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    import ctypes

    import numpy as np
    import torch
    import torch.distributed as dist

    from ray_tracer_fragment_shader_amd import abi, scenes
    from ray_tracer_fragment_shader_amd.distributed import BandPlan, assemble_on_device, exchange_frames
    from ray_tracer_fragment_shader_amd.tracer import Tracer

    if not torch.cuda.is_available():
        print("bench.py needs a HIP GPU", file=sys.stderr)
        return 2
    ndev = torch.cuda.device_count()
    if world > 1 and args.backend == "nccl" and ndev < world:
        print(f"bench.py: {world} ranks with the nccl (RCCL) backend need {world} GPUs, this host shows {ndev} "
              f"(rehearse with --backend gloo)", file=sys.stderr)
        return 2
    rehearsal = args.backend == "gloo" and ndev == 1
    if rehearsal:
        local = 0                                           # rehearsal: all ranks share the one GPU
    torch.cuda.set_device(local)
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
    L = abi.lib()
    dev = torch.device("cuda", local)
    # Every leg runs on ordinary (non-null) streams: the legacy null stream's implicit ordering cost the c2 frames in
    # flight 26.4 us per frame against 23.8 on three pool streams, and 0.7 us per serial launch (tools/c4_gap_probe.py
    # part 3, BENCH_r05).  This process's current stream becomes one, so torch work stays ordered with it.
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    # the frames-in-flight streams, created right after the bench's stream and before any context creates its own:
    # HIP hands out its four hardware queues in creation order, so streams created together get distinct queues
    # (created later, one shared the bench stream's queue: the moving-camera leg ran 28.2 against 23.0 us per frame)
    frame_streams(torch, dev, stream, max(1, args.frames_in_flight))

    def barrier():
        if world > 1:
            dist.barrier()

    def max_over_ranks(x: float) -> float:
        if world == 1:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=dev if args.backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def fail_together(msg):
        """Every rank reaches this with its own msg (None: fine); if any rank failed, all exit non-zero together
        (one rank leaving alone would leave its peers blocked in the next collective)."""
        bad = 0.0 if msg is None else 1.0
        if max_over_ranks(bad) > 0.0:
            raise SystemExit(msg or f"parity failure on another rank (this is rank {rank})")

    def frame_rays(tr, cam, W, H, B):
        b = tr.render(cam, W, H, B, rgba32f=False, raycount=True)
        torch.cuda.synchronize()
        rc = b["raycount"].view(torch.int32)
        return int((rc & 0xFFFF).sum().item()) + int((rc >> 16).sum().item())

    # ---- one frame split over all ranks, RCCL gather to rank 0 (C ABI group) ----------------------------
    def group_leg(cfg, steps, warmup, copy_ranks=0):
        """rt_render_multi over the job's ranks (one process per GPU: rt_group_create_rank; N = 1: a
        one-rank RCCL group).  copy_ranks > 0 (gloo rehearsal on one GPU, rank 0 only): one process driving
        `copy_ranks` contexts that share the device, COPY transport — the same group code, no xGMI.
        Returns (stats dict, seconds for `steps` frames, max over ranks)."""
        W, H, B = cfg.width, cfg.height, cfg.depth
        cam = cfg.camera()
        t = Tracer(local)
        t.set_scene(cfg.scene())
        g = ctypes.c_void_p()
        extra = []
        if copy_ranks:
            extra = [Tracer(local) for _ in range(copy_ranks - 1)]
            for e in extra:
                e.set_scene(cfg.scene())
            arr = (ctypes.c_void_p * copy_ranks)(t._ctx.value, *[e._ctx.value for e in extra])
            abi.check(L.rt_group_create(arr, copy_ranks, abi.RT_TRANSPORT_COPY, ctypes.byref(g)), "rt_group_create")
        elif world > 1:
            idt = torch.zeros(abi.RT_COMM_ID_BYTES, dtype=torch.uint8)
            if rank == 0:
                abi.check(L.rt_comm_unique_id(ctypes.c_void_p(idt.data_ptr())), "rt_comm_unique_id")
            idd = idt.to(dev) if args.backend == "nccl" else idt
            dist.broadcast(idd, 0)
            idt = idd.cpu()
            abi.check(L.rt_group_create_rank(t._ctx, world, rank, ctypes.c_void_p(idt.data_ptr()), ctypes.byref(g)),
                      "rt_group_create_rank")
        else:
            arr = (ctypes.c_void_p * 1)(t._ctx.value)
            abi.check(L.rt_group_create(arr, 1, abi.RT_TRANSPORT_RCCL, ctypes.byref(g)), "rt_group_create")
        gw = copy_ranks or world                           # ranks of the group
        gp = abi.rt_group_plan()                           # the group's frame plan (rank 0's view of it)
        abi.check(L.rt_group_plan_frame(W, H, gw, 0, args.band_height, abi.RT_OUT_RGBA8, 1, ctypes.byref(gp)),
                  "rt_group_plan_frame")
        img8 = torch.empty((H, W, 4), dtype=torch.uint8, device=dev) if rank == 0 else None
        argv = (g, ctypes.byref(cam), W, H, B, args.band_height, abi.RT_OUT_RGBA8,
                None, ctypes.c_void_p(img8.data_ptr()) if img8 is not None else None, ctypes.c_void_p(stream.cuda_stream))
        fn = L.rt_render_multi

        def sync():
            abi.check(L.rt_group_synchronize(g), "rt_group_synchronize")
            torch.cuda.synchronize()

        # untimed: the tile-order calibration of every rank, then frames until the clocks have ramped up — a fixed
        # count on every rank (each frame is a collective), SETTLE_FRAMES_PER_S per second of --settle (BENCH_r05's
        # one-rank frame, timed after the 20 warm-up frames alone, was 14% slower than settled: tools/c4_gap_probe.py)
        for _ in range(max(warmup, 20) + settle_frames(args.settle)):
            abi.check(fn(*argv), "rt_render_multi")
        sync()
        if not copy_ranks:
            barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            rc = fn(*argv)
            if rc:
                abi.check(rc, "rt_render_multi")
        sync()
        if not copy_ranks:
            barrier()
        elapsed = time.perf_counter() - t0 if copy_ranks else max_over_ranks(time.perf_counter() - t0)
        # per-phase times (HIP events on the group's render / comm streams), in a separate untimed pass so the
        # events do not perturb the timed one
        abi.check(L.rt_group_timing(g, 1), "rt_group_timing")
        for _ in range(min(steps, 32)):
            abi.check(fn(*argv), "rt_render_multi")
        st = abi.rt_group_stats()
        abi.check(L.rt_group_get_stats(g, ctypes.byref(st)), "rt_group_get_stats")
        torch.cuda.synchronize()
        if not copy_ranks:
            barrier()
        phases = {"render_ms": st.render_ms, "gather_ms": st.gather_ms, "assemble_ms": st.assemble_ms,
                  "frame_ms": st.frame_ms}
        phases_max = ({k: round(v, 5) for k, v in phases.items()} if copy_ranks else
                      {k: round(max_over_ranks(v), 5) for k, v in phases.items()})
        names = {abi.RT_PIXEL_GRAY8: "GRAY8", abi.RT_PIXEL_RGB8: "RGB8", abi.RT_PIXEL_RGBA8: "RGBA8", -1: None}
        parity = None
        if rank == 0:                                      # gathered frame == one-launch frame, every byte
            ref = t.render(cam, W, H, B, rgba32f=False, rgba8=True)["rgba8"]
            torch.cuda.synchronize()
            parity = bool(torch.equal(ref, img8))
        rays = frame_rays(t, cam, W, H, B) if rank == 0 else 0
        L.rt_group_destroy(g)
        t.close()
        for e in extra:
            e.close()
        info = {"ranks": gw, "rccl_world": 0 if copy_ranks else world,
                "transport": "COPY (rehearsal: contexts share one GPU)" if copy_ranks else "RCCL",
                "band_height": gp.band_height, "slab_rows": gp.slab_rows, "renderers": gp.renderers,
                "root_renders": bool(gp.root_renders), "rays_per_frame": rays, "parity": parity,
                "wire_format": names.get(st.wire_byte, st.wire_byte), "payload_bytes_to_rank0": st.payload_bytes,
                "phases_ms_rank0": {k: round(v, 5) for k, v in phases.items()} if rank == 0 else None,
                "phases_ms_max_over_ranks": phases_max,
                "phases_note": "HIP events on each rank's render / comm streams over min(steps, 32) untimed frames: "
                               "render = rt_render_dev of the rank's bands; gather = from the rank's render end to its "
                               "ncclSend done (rank > 0), or from the frame's hand-off to every ncclRecv done (rank 0: "
                               "its receives are posted without waiting for its own render; includes waiting for peers); "
                               "assemble = rank 0's unshuffle + expand into RGBA8; frame = rank 0 render start to "
                               "assembled image (frames overlap: double-buffered slabs)"}
        if parity is False:
            info["error"] = "gathered RGBA8 frame differs from the one-launch frame"
        return info, elapsed

    cfg = scenes.CONFIGS[args.config]
    W, H, B = cfg.width, cfg.height, cfg.depth
    scene = cfg.scene()
    cam = cfg.camera()
    streams = world > 1 and args.scaling == "streams"       # banded frames + all-to-all
    strong = world > 1 and args.scaling == "strong"         # one banded frame + RCCL gather (C ABI group)
    if strong and rehearsal:
        raise SystemExit("--scaling strong needs one GPU per rank (RCCL refuses two ranks on one device)")
    parity = "skipped"
    res_extra = {}

    if strong:
        info, elapsed = group_leg(cfg, args.steps, args.warmup)
        rays_frame = info["rays_per_frame"]
        job_frames = 1
        # the kernel alone on this rank's rows (the first renderer's when rank 0 only assembles), for the roofline
        nr, ri = info["renderers"], rank if info["root_renders"] else max(rank - 1, 0)
        plan = BandPlan(H, nr, info["band_height"])
        nl = plan.frame_local[ri]
        tr = Tracer(local)
        tr.set_scene(scene)
        bufs = tr.alloc(W, H, plan.rows(ri), rgba32f=True, rgba8=True)
        for _ in range(3):
            tr.render_into(cam, W, H, B, bufs, rows=plan.rows(ri))
        e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        torch.cuda.synchronize()
        e[0].record(stream)
        for _ in range(20):
            tr.render_into(cam, W, H, B, bufs, rows=plan.rows(ri))
        e[1].record(stream)
        torch.cuda.synchronize()
        avg_kern_ms = kern_serial_ms = e[0].elapsed_time(e[1]) / 20
        nfly = 1
        fail_together("parity failure: the gathered RGBA8 frame differs from the one-launch frame"
                      if rank == 0 and not info["parity"] else None)
        parity = f"gathered RGBA8 frame == one-launch frame: {info['parity']}"
        res_extra["group"] = info
    else:
        tr = Tracer(local)
        tr.set_scene(scene)
        frames = world if streams else 1                    # frames stacked in one launch on this rank
        job_frames = world
        plan = BandPlan(H, world if streams else 1, args.band_height, frames=frames)
        if streams and not plan.balanced:
            raise SystemExit(f"frame streams need equal rows per rank: H={H}, N={world}, band {plan.band_height}")
        prank = rank if streams else 0
        rows = plan.rows(rank) if streams else None
        nl = plan.local[prank]                 # rows this rank renders per step (all its frames)
        fl = plan.frame_local[prank]           # ... per frame

        # ---- parity + ray count (outside the timed region) ----------------------------------------------
        rays_frame = scenes.PINNED_RAYS.get(args.config)
        if not args.profile_kernel_only:
            chk = tr.render(cam, W, H, B, rgba32f=False, rgb64f=True, raycount=True)
            torch.cuda.synchronize()
            rc = chk["raycount"].cpu().numpy().view(np.uint32)
            rays_frame = int((rc & 0xFFFF).sum()) + int((rc >> 16).sum())
            pinned = scenes.PINNED_RAYS.get(args.config)
            g = np.load(os.path.join(ROOT, "tests", "golden", f"frames_{args.config}.npz"))
            got = chk["rgb64f"].cpu().numpy()[g["pj"], g["pi"]]
            fail_together(f"ray count {rays_frame} != reference {pinned}" if pinned is not None and rays_frame != pinned
                          else None if np.array_equal(got, g["samples"]) else
                          f"parity failure: max err {np.abs(got - g['samples']).max()}")
            parity = "bit-exact on 4096 sampled pixels vs the reference's rayTraceRay (tests/golden)"
            del chk, rc

        fn = L.rt_render_dev
        if not streams:
            # Independent frames: frame s goes to stream s % F with its own context and output buffers, so its
            # launch fills the tail of frame s-1 (F = --frames-in-flight).  Every frame is a full render.
            nfly = max(1, args.frames_in_flight)
            trs = [tr] + [Tracer(local) for _ in range(nfly - 1)]
            for t in trs[1:]:
                t.set_scene(scene)
            sts = frame_streams(torch, dev, stream, nfly)                              # (pool streams, not null)
            outs = [(torch.empty((nl, W, 4), dtype=torch.float32, device=dev),
                     torch.empty((nl, W, 4), dtype=torch.uint8, device=dev)) for _ in range(nfly)]
            launch_args = [(trs[i]._ctx, ctypes.byref(cam), W, H, B, None, ctypes.c_void_p(outs[i][0].data_ptr()),
                            ctypes.c_void_p(outs[i][1].data_ptr()), None, None, ctypes.c_void_p(sts[i].cuda_stream))
                           for i in range(nfly)]
            # Setup (untimed): per context, the first render of the view uses the identity tile order, the
            # second times its tile rows (calibration), later renders dispatch the longest rows first; then
            # --settle seconds of frames and the --warmup steps, untimed.
            for _ in range(2):
                for la in launch_args:
                    abi.check(fn(*la), "rt_render_dev")
            torch.cuda.synchronize()
            wsteps = max(args.warmup, 0)
            for i in range(wsteps):
                abi.check(fn(*launch_args[i % nfly]), "rt_render_dev")
            torch.cuda.synchronize()
            barrier()
            elapsed, avg_kern_ms = pipelined_frames(torch, L, abi, trs, sts, launch_args, args.steps, args.settle)
            barrier()
            # (skipped in --profile-kernel-only runs, whose trace must end with the timed dispatches)
            kern_serial_ms = (None if args.profile_kernel_only else
                              serial_kernel_ms(torch, L, abi, launch_args[0], stream))
            elapsed = max_over_ranks(elapsed)
            for t in trs[1:]:
                t.close()
        else:
            out32 = torch.empty((nl, W, 4), dtype=torch.float32, device=dev)
            # RGBA8 slabs are double-buffered: a step's exchange reads them while the next step renders
            out8 = [torch.empty((nl, W, 4), dtype=torch.uint8, device=dev) for _ in range(2)]
            recv8 = [torch.empty((world, fl, W, 4), dtype=torch.uint8, device=dev) for _ in range(2)]
            image8 = [torch.empty((H, W, 4), dtype=torch.uint8, device=dev) for _ in range(2)]
            side = torch.cuda.Stream(dev)
            assembled = [torch.cuda.Event() for _ in range(2)]
            pending = [None, None]
            nfly = 1
            # Pre-bound launches: the ctypes argument tuples are built once, so the timed loop only issues
            # rt_render_dev (host cost ~8 us per call; the GPU queue stays full).
            rows_ref = ctypes.byref(rows)
            launch_args = [(tr._ctx, ctypes.byref(cam), W, H, B, rows_ref, ctypes.c_void_p(out32.data_ptr()),
                            ctypes.c_void_p(out8[b].data_ptr()), None, None, ctypes.c_void_p(stream.cuda_stream))
                           for b in range(2)]
            counter = [0]

            def step():
                b = counter[0] % 2
                counter[0] += 1
                if pending[b] is not None:
                    pending[b].wait()                           # the all-to-all of step s-2 has read out8[b]
                rc = fn(*launch_args[b])
                if rc:
                    abi.check(rc, "rt_render_dev")
                stream.wait_event(assembled[b])                 # recv8[b] consumed by the assembly of step s-2
                pending[b] = exchange_frames(out8[b].view(world, fl, W, 4), recv8[b], world, async_op=True)
                with torch.cuda.stream(side):
                    if pending[b] is not None:
                        pending[b].wait()
                    else:                                       # host-staged rehearsal: recv8[b] filled on `stream`
                        side.wait_stream(stream)
                    assemble_on_device(recv8[b], plan, W, image8[b], side)
                    assembled[b].record(side)

            for _ in range(2):
                for la in launch_args:
                    abi.check(fn(*la), "rt_render_dev")
            torch.cuda.synchronize()
            for _ in range(args.warmup):
                step()
            barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                step()
            torch.cuda.synchronize()                            # every stream: render, exchange, assembly
            barrier()
            elapsed = time.perf_counter() - t0
            # the timed region also holds the exchange: time the kernel alone in a short post-pass
            avg_kern_ms = kern_serial_ms = serial_kernel_ms(torch, L, abi, launch_args[0], stream)
            elapsed = max_over_ranks(elapsed)

    rays_step = rays_frame * job_frames
    value = rays_step * args.steps / elapsed / 1e6
    ms_step = elapsed / args.steps * 1e3
    # The roofline divides by the kernel's own launch duration: launches back to back on one stream (HIP events
    # on that stream), the figure a one-stream rocprofv3 kernel trace reports as AverageNs (profiles/).  The
    # per-frame interval with frames in flight (shorter: a launch fills the previous one's tail) is reported
    # beside it.
    launch_ms = kern_serial_ms if kern_serial_ms is not None else avg_kern_ms
    roof, roof64 = kernel_rooflines(args.config, nl, W, H, launch_ms)
    roof["kernel_ms_serial"] = round(kern_serial_ms, 5) if kern_serial_ms is not None else None
    roof["interval_ms_in_flight"] = round(avg_kern_ms, 5)
    roof["frames_in_flight"] = nfly
    roof["kernel_ms_note"] = ("kernel_ms = kernel_ms_serial: average duration of rt_render_kernel launched back to "
                              "back on one stream (HIP events on that stream); interval_ms_in_flight: per-frame "
                              f"interval over the timed region with {nfly} launch stream(s), HIP events bracketing "
                              "them (a frame's launch overlaps the previous frame's tail when > 1)")
    prof = rocprof_reference(args.config, nl == H and world == 1)
    if prof:
        roof.update(prof)
        # the committed profile's frac, and its agreement with the live launch duration
        roof["frac_rocprof"] = round(roof["achieved"] * launch_ms / (prof["rocprof_avg_us"] / 1e3) / roof["peak"], 5)
        roof["rocprof_vs_live"] = round(prof["rocprof_avg_us"] / 1e3 / launch_ms, 4)
    if world > 1:
        roof["traffic"] = None                               # the PMC figures are whole-frame, one GPU

    # ---- extra legs (outside the timed region of `value`) --------------------------------------------------
    extra_ok = not args.profile_kernel_only

    def result():
        """The JSON line (rank 0): the timed metric above plus the extra legs gathered so far."""
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
                                f"row bands (h={plan.band_height}) x {world} ranks + RCCL gather to rank 0 "
                                f"(rt_render_multi)" if strong else
                                f"{world} ranks x whole frames (independent frames, no collective)"
                                + c4_parallelism_text(world, res_extra.get("c4"))
                                if world > 1 else "single GPU"),
            },
            "roofline": roof,
            "roofline_fp64": roof64,
            "parity": parity,
        }
        res.update(res_extra)
        return res

    if extra_ok and not args.no_c4 and not strong:
        # Guarded: the timed metric above is already final.  A failure of this leg is reported in its
        # entry; a leg that does not finish within --c4-timeout seconds (e.g. a peer that never joins the
        # RCCL gather) ends the job with the line as it stands rather than leaving it without one, and with
        # exit code 3, so the hang is not read as success.
        import threading

        def c4_timeout():
            if rank == 0:
                res_extra["c4"] = {"error": f"c4 leg did not finish within {args.c4_timeout:g} s"}
                print(json.dumps(result()), file=out, flush=True)
            os._exit(3)                                     # the line stands, the job did not finish: non-zero

        dog = threading.Timer(args.c4_timeout, c4_timeout)
        dog.daemon = True
        dog.start()
        try:
            c3 = scenes.CONFIGS["c3"]
            steps4 = 40                                    # (fixed: the first launch and the final sync weigh less)
            # the denominator of the split frame's speed-up: the same job's one-GPU c3 frame (same scene, view and
            # RGBA8 output), measured on rank 0 before the group leg at every N
            base = (c3_one_gpu(torch, L, abi, Tracer, c3, dev, local, max(1, args.frames_in_flight), steps4,
                               args.settle) if rank == 0 else None)
            barrier()
            if rehearsal:                                   # gloo on one GPU: rank 0 drives `world` COPY ranks
                info, el4 = group_leg(c3, steps4, 3, copy_ranks=world) if rank == 0 else ({}, 0.0)
                barrier()
            else:
                info, el4 = group_leg(c3, steps4, 3)
            info.update({"workload": "c4: c3's 3840x2160 frame (8 spheres + board, 2 lights, 2 bounces) split "
                                     f"over {world} rank(s) in round-robin row bands, RGBA8 gathered to rank 0 over "
                                     "RCCL (ncclSend/ncclRecv in rt_render_multi) and unshuffled there"
                                     if world > 1 else
                                     "c4 machinery at one rank: c3's 3840x2160 frame through rt_render_multi of a "
                                     "one-rank RCCL group (identity band plan: rendered straight into the image)",
                         "frames": steps4, "ms_per_frame": round(el4 / steps4 * 1e3, 4) if el4 else None,
                         "value": (round(info["rays_per_frame"] * steps4 / el4 / 1e6, 3)
                                   if rank == 0 and "error" not in info else None),
                         "unit": "Mray/s", "scaling": "strong"})
            if rank == 0 and base and "error" not in info:
                info.update(c4_scaling_keys(info["ranks"], c3.width, c3.height, info["rays_per_frame"],
                                            el4 / steps4 * 1e3, *base))
                if world == 1:                              # what one GPU says about 2, 4 and 8 ranks
                    proj = {}
                    for n in (2, 4, 8):
                        proj.update(c4_rank_projection(torch, L, abi, Tracer, c3, dev, local, n, args.band_height,
                                                       base[0]))
                    proj["note"] = ("one-GPU projection of the c4 frame at n ranks (rt_render_multi at n > 1 needs n "
                                    "GPUs): nN_rank_render_ms = each renderer's band set rendered alone as the group "
                                    "renders it (GRAY8 slab, two render streams taking frames in turn; from 4 ranks the "
                                    "renderers are ranks 1 .. n-1 and rank 0 only assembles, nN_root_renders); "
                                    "nN_rank0_ms = rank 0's pipeline as the group runs it (its bands if it renders, "
                                    "then per frame the unpack of the gathered GRAY8 buffer into RGBA8 on its comm "
                                    "stream beside the next render, 3 frame buffers); nN_projected_frame_ms = the "
                                    "slowest of rank 0 and the peers (or the "
                                    "nominal xGMI gather of one slab if longer); nN_speedup_bound = "
                                    "c3_1gpu_ms_per_frame / nN_projected_frame_ms")
                    info["projection"] = proj
                info["scaling_note"] = ("speedup_vs_c3_1gpu = c3_1gpu_ms_per_frame (one GPU, RGBA8 only, "
                                        f"{max(1, args.frames_in_flight)} frames in flight, measured on rank 0 of this "
                                        "job before the group leg) / ms_per_frame; efficiency = speedup / ranks; "
                                        "hbm_write_frac_per_gpu = (W x H x 4 B / ranks) / ms_per_frame / 8 TB/s")
            res_extra["c4"] = info
        except Exception as exc:                            # reported, the timed metric stands
            res_extra["c4"] = {"error": f"{type(exc).__name__}: {exc}"}
        dog.cancel()

    if rank == 0 and world == 1 and extra_ok and not args.no_extra:
        confs = {}
        for name, k in (("c3", 40), ("c5", 16)):
            c = scenes.CONFIGS[name]
            t = Tracer(local)
            t.set_scene(c.scene())
            cc = c.camera()
            rays = frame_rays(t, cc, c.width, c.height, c.depth)
            if rays != scenes.PINNED_RAYS[name]:
                raise SystemExit(f"{name}: ray count {rays} != reference {scenes.PINNED_RAYS[name]}")
            nf = max(1, args.frames_in_flight)
            ts = [t] + [Tracer(local) for _ in range(nf - 1)]
            for tt in ts[1:]:
                tt.set_scene(c.scene())
            ss = frame_streams(torch, dev, stream, nf)
            bb = [tt.alloc(c.width, c.height, rgba32f=True, rgba8=True) for tt in ts]
            la = [(ts[i]._ctx, ctypes.byref(cc), c.width, c.height, c.depth, None,
                   ctypes.c_void_p(bb[i]["rgba32f"].data_ptr()), ctypes.c_void_p(bb[i]["rgba8"].data_ptr()), None,
                   None, ctypes.c_void_p(ss[i].cuda_stream)) for i in range(nf)]
            for _ in range(2):
                for a in la:
                    abi.check(L.rt_render_dev(*a), "rt_render_dev")
            wall, kms = pipelined_frames(torch, L, abi, ts, ss, la, k, min(args.settle, 0.1))
            wall /= k
            kser = serial_kernel_ms(torch, L, abi, la[0], stream, n=max(5, k // 2))
            for tt in ts[1:]:
                tt.close()
            r1, r2 = kernel_rooflines(name, c.height, c.width, c.height, kser)
            confs[name] = {"workload": f"{name}: {c.width}x{c.height}, {c.n_spheres} spheres + board, "
                                       f"{c.n_lights} light(s), {c.depth} bounce(s), one GPU",
                           "ms_per_frame": round(wall * 1e3, 4), "value": round(rays / wall / 1e6, 3),
                           "unit": "Mray/s", "rays_per_frame": rays, "kernel_ms": round(kser, 5),
                           "kernel_ms_serial": round(kser, 5), "interval_ms_in_flight": round(kms, 5),
                           "frames_in_flight": nf,
                           "hbm_frac": r1["frac"], "hbm_traffic": r1["traffic"],
                           "algorithmic_bytes": r1["algorithmic_bytes_per_launch"], "fp64_frac": r2["frac"],
                           "fp64_reference_equivalent_tflops": r2["reference_equivalent_tflops"]}
            prof = rocprof_reference(name, True)
            if prof:
                confs[name].update(prof)
                confs[name]["hbm_frac_rocprof"] = round(
                    r1["algorithmic_bytes_per_launch"] / (prof["rocprof_avg_us"] * 1e-6) / 1e9 / r1["peak"], 5)
                confs[name]["rocprof_vs_live"] = round(prof["rocprof_avg_us"] / 1e3 / kser, 4)
            t.close()
        res_extra["configs"] = confs

        # draw()'s replacement: rt_render (host buffers, synchronous) every frame at c2, RGBA8 back to the host
        di = {}
        sa = scene.to_abi()
        host8 = torch.empty((H, W, 4), dtype=torch.uint8).pin_memory()
        t = Tracer(local)
        args_r = (t._ctx, ctypes.byref(sa), ctypes.byref(cam), W, H, B, None, None,
                  ctypes.c_void_p(host8.data_ptr()), None, None)
        for _ in range(3):
            abi.check(L.rt_render(*args_r), "rt_render")
        k = 30
        t0c = time.perf_counter()
        for _ in range(k):
            abi.check(L.rt_render(*args_r), "rt_render")
        di["rt_render_ms_per_call"] = round((time.perf_counter() - t0c) / k * 1e3, 4)
        di["rt_render_note"] = ("c2 frame, RGBA8 (8.3 MB) copied to pinned host memory each call; scene upload "
                                "skipped (unchanged); includes launch, kernel, PCIe copy and synchronisation")
        di.update(packed_host_legs(t, sa, cam, W, H, B))
        di["dropin_binding"] = dropin_binding_legs(W, H, B, cfg)
        # moving camera: a new eye every frame (per-eye preparation every frame; each new view in identity tile
        # order), frames in flight as in the static leg
        views = []
        for v in range(16):
            c2 = cfg.camera()
            ang = 2.0 * np.pi * v / 16
            c2.eye = abi.vec3((60.0 * np.sin(ang), 100.0 + 10.0 * np.cos(ang), 200.0))
            views.append(c2)
        t.set_scene(scene)
        mrays = [frame_rays(t, v, W, H, B) for v in views]
        nf = max(1, args.frames_in_flight)
        ts = [t] + [Tracer(local) for _ in range(nf - 1)]
        for tt in ts[1:]:
            tt.set_scene(scene)
        # (streams of their own: on the streams that had run the static legs' frames the same moving frames measured
        # 28.2 against 23.0 us per frame — cause not found; in a fresh process either kind measures 23 us,
        # tools/moving_probe.py)
        ss = [torch.cuda.Stream(dev) for _ in range(nf)]
        bb = [tt.alloc(W, H, rgba32f=True, rgba8=True) for tt in ts]
        nla = 16 * nf                                      # frame i: view i % 16 on stream i % nf
        la = [(ts[i % nf]._ctx, ctypes.byref(views[i % 16]), W, H, B, None,
               ctypes.c_void_p(bb[i % nf]["rgba32f"].data_ptr()), ctypes.c_void_p(bb[i % nf]["rgba8"].data_ptr()),
               None, None, ctypes.c_void_p(ss[i % nf].cuda_stream)) for i in range(nla)]
        k = 96                                             # median of three passes (the clocks settled first)
        passes = [pipelined_frames(torch, L, abi, ts, ss, la, k, min(args.settle, 0.3) if p == 0 else 0.0)
                  for p in range(3)]
        walls = [w / k for w, _ in passes]
        wall = sorted(walls)[1]
        di["moving_camera"] = {"ms_per_frame": round(wall * 1e3, 4),
                               "value": round(sum(mrays) / 16 / wall / 1e6, 3),
                               "unit": "Mray/s", "static_view_ms_per_frame": round(ms_step, 4),
                               "frames_in_flight": nf,
                               "passes_ms_per_frame": [round(w * 1e3, 4) for w in walls],
                               "interval_ms_in_flight": round(sorted(x for _, x in passes)[1], 4),
                               "note": "c2 scene, eye moves on a 16-view orbit, every frame a new eye "
                                       "(rt_prepare_kernel each frame, primary cone masks in the kernel, each new "
                                       "view in identity tile order — r06; RT_MOVING_ORDER=1 reuses the last "
                                       "calibrated order); median of three passes of 96 frames"}
        for tt in ts[1:]:
            tt.close()
        t.close()
        res_extra["drop_in"] = di

    if rank == 0:
        res = result()
        if world == 1 and not args.no_cpu_baseline and not args.profile_kernel_only:
            res["cpu_baseline"] = cpu_baseline(args, cfg, scene, cam, W, H, B, rays_frame)
        print(json.dumps(res), file=out, flush=True)
    tr.close()
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
