#!/usr/bin/env python3
"""Why the bench's one-rank c4 frame (rt_render_multi, 0.1332 ms in BENCH_r05) is slower than the same job's serial c3
frame (0.1163 ms) while tools/c4_n1_probe.py, which keeps the GPU busy between modes, measures them equal; and what
one GPU says about an 8-rank c4 frame.

Part 1 (cold vs settled): the bench's group-leg procedure (20 untimed frames, 40 timed by the wall clock) started
after the GPU idled for IDLE_S seconds, against the same procedure after SETTLE_S seconds of back-to-back frames.
Modes: the one-rank group on the null stream (the bench), on a non-blocking stream, and plain rt_render_dev.

Part 2 (N-rank projection): for N in 2, 4, 8, each rank's band set (rt_rows(hb, N, r)) rendered alone as GRAY8 into
its slab, back to back on one stream and alternating over two streams (frames of the same rank overlapping), and
rank 0's rt_unpack_dev of an N-rank gathered GRAY8 buffer into the RGBA8 image.  Prints JSON lines."""
import ctypes
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from ray_tracer_fragment_shader_amd import abi, scenes  # noqa: E402
from ray_tracer_fragment_shader_amd.tracer import Tracer  # noqa: E402

L = abi.lib()
cfg = scenes.CONFIGS["c3"]
W, H, B = cfg.width, cfg.height, cfg.depth
cam = cfg.camera()


def settle(fn, seconds):
    t_end = time.perf_counter() + seconds
    while time.perf_counter() < t_end:
        for _ in range(16):
            abi.check(fn(), "settle")
        torch.cuda.synchronize()


def wall_ms(fn, n, sync):
    sync()
    t0 = time.perf_counter()
    for _ in range(n):
        rc = fn()
        if rc:
            abi.check(rc, "timed")
    sync()
    return (time.perf_counter() - t0) * 1e3 / n


def event_ms(fn, n, stream):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record(stream)
    for _ in range(n):
        abi.check(fn(), "timed")
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


def part1(rounds):
    null = torch.cuda.current_stream()
    nb = torch.cuda.Stream()
    t_multi, t_dev = Tracer(0), Tracer(0)
    for t in (t_multi, t_dev):
        t.set_scene(cfg.scene())
    img = torch.empty((H, W, 4), dtype=torch.uint8, device="cuda")
    g = ctypes.c_void_p()
    arr = (ctypes.c_void_p * 1)(t_multi._ctx.value)
    abi.check(L.rt_group_create(arr, 1, abi.RT_TRANSPORT_RCCL, ctypes.byref(g)), "rt_group_create")

    def multi(st):
        return lambda: L.rt_render_multi(g, ctypes.byref(cam), W, H, B, 0, abi.RT_OUT_RGBA8, None,
                                         ctypes.c_void_p(img.data_ptr()), ctypes.c_void_p(st.cuda_stream))

    def dev(st):
        return lambda: L.rt_render_dev(t_dev._ctx, ctypes.byref(cam), W, H, B, None, None,
                                       ctypes.c_void_p(img.data_ptr()), None, None, ctypes.c_void_p(st.cuda_stream))

    def gsync():
        abi.check(L.rt_group_synchronize(g), "rt_group_synchronize")
        torch.cuda.synchronize()

    modes = {"multi_null": multi(null), "multi_nonblocking": multi(nb), "dev_null": dev(null)}
    res = {f"{m}_{k}": [] for m in modes for k in ("cold", "settled")}
    idle, sett = float(os.environ.get("IDLE_S", "1.0")), float(os.environ.get("SETTLE_S", "0.25"))
    for f in modes.values():
        for _ in range(3):
            abi.check(f(), "first renders")
    torch.cuda.synchronize()
    for _ in range(rounds):
        for m, f in modes.items():
            time.sleep(idle)
            for _ in range(20):
                abi.check(f(), "warm")
            res[f"{m}_cold"].append(wall_ms(f, 40, gsync))
            settle(f, sett)
            for _ in range(20):
                abi.check(f(), "warm")
            res[f"{m}_settled"].append(wall_ms(f, 40, gsync))
    out = {k: round(statistics.median(v), 5) for k, v in res.items()}
    out["dev_null_event_ms_serial"] = round(event_ms(modes["dev_null"], 40, null), 5)
    print(json.dumps({"part": 1, "config": "c3", "idle_s": idle, "settle_s": sett, "rounds": rounds,
                      "wall_ms_per_frame": out}), flush=True)
    L.rt_group_destroy(g)
    t_multi.close()
    t_dev.close()


def part2(ns):
    """Per rank r of n: its band set rendered alone as GRAY8, serial (one stream) and with K streams taking frames in
    turn (K = 2, 3: frames of the same rank overlapping, the group's double / triple buffering), for each band height
    in HBS (0: rt_band_plan's choice); rank 0's rt_unpack_dev of an n-rank gathered GRAY8 buffer."""
    t = Tracer(0)
    t.set_scene(cfg.scene())
    st = [torch.cuda.Stream() for _ in range(3)]
    img = torch.empty((H, W, 4), dtype=torch.uint8, device="cuda")
    full = lambda: L.rt_render_dev(t._ctx, ctypes.byref(cam), W, H, B, None, None, ctypes.c_void_p(img.data_ptr()),  # noqa
                                   None, None, ctypes.c_void_p(st[0].cuda_stream))
    settle(full, 0.3)
    c3_serial = event_ms(full, 40, st[0])
    for n in ns:
        for hb_req in [int(x) for x in os.environ.get("HBS", "0,8").split(",")]:
            band, slab = ctypes.c_int(), ctypes.c_int()
            abi.check(L.rt_band_plan(H, n, hb_req, ctypes.byref(band), ctypes.byref(slab)), "rt_band_plan")
            hb, sr = band.value, slab.value
            ranks = []
            trs = [Tracer(0) for _ in range(n)]             # one context per rank: its own view (rows) calibration
            for r in range(n):
                trs[r].set_scene(cfg.scene())
                rows = abi.rt_rows(hb, n, r, 1)
                slabs = [torch.empty((sr, W), dtype=torch.uint8, device="cuda") for _ in range(3)]

                def one(b, rows=rows, slabs=slabs, tr=trs[r]):
                    return L.rt_render_dev_packed(tr._ctx, ctypes.byref(cam), W, H, B, ctypes.byref(rows),
                                                  abi.RT_PIXEL_GRAY32F, None, abi.RT_PIXEL_GRAY8,
                                                  ctypes.c_void_p(slabs[b].data_ptr()), ctypes.c_void_p(st[b].cuda_stream))
                for b in range(3):
                    for _ in range(3):                       # first render + calibration of this view (rows)
                        abi.check(one(b), "first")
                torch.cuda.synchronize()
                rec = {"rank": r}
                settle(full, 0.05)
                rec["serial_ms"] = round(event_ms(lambda one=one: one(0), 40, st[0]), 5)
                for k in (2, 3):
                    cnt = [0]

                    def alt(one=one, cnt=cnt, k=k):
                        cnt[0] += 1
                        return one(cnt[0] % k)
                    settle(full, 0.05)
                    rec[f"streams{k}_ms"] = round(wall_ms(alt, 120, torch.cuda.synchronize), 5)
                ranks.append(rec)
            gathered = torch.zeros((n * sr, W), dtype=torch.uint8, device="cuda")
            up = lambda: L.rt_unpack_dev(ctypes.c_void_p(gathered.data_ptr()), ctypes.c_void_p(img.data_ptr()), W, H,  # noqa
                                         abi.RT_PIXEL_GRAY8, abi.RT_PIXEL_RGBA8, hb, n, sr,
                                         ctypes.c_void_p(st[0].cuda_stream))
            for _ in range(5):
                abi.check(up(), "unpack")
            unpack = event_ms(up, 40, st[0])
            out = {"part": 2, "n": n, "band_height": hb, "slab_rows": sr, "c3_serial_ms": round(c3_serial, 5),
                   "unpack_ms": round(unpack, 5), "ranks": ranks}
            for key in ("serial_ms", "streams2_ms", "streams3_ms"):
                m = max(x[key] for x in ranks)
                out["max_" + key] = m
                out["bound_" + key] = round(c3_serial / (m + unpack), 3)
            print(json.dumps(out), flush=True)
            for x in trs:
                x.close()
    t.close()


def hip_runtime():
    """The HIP runtime already loaded in this process (torch's or /opt/rocm's), by its path in /proc/self/maps."""
    with open("/proc/self/maps") as f:
        for line in f:
            if "libamdhip64.so" in line:
                return ctypes.CDLL(line.split()[-1])
    raise RuntimeError("no libamdhip64 loaded")


def make_streams(kind, k):
    """k streams: torch's pool ("torch"), fresh non-blocking HIP streams ("hip"), or HIP streams with a full CU mask
    ("cumask": a queue of their own in ROCclr)."""
    hip = hip_runtime()
    out = []
    for _ in range(k):
        h = ctypes.c_void_p()
        if kind == "hip":
            rc = hip.hipStreamCreateWithFlags(ctypes.byref(h), 1)
        else:
            mask = (ctypes.c_uint32 * 8)(*([0xFFFFFFFF] * 8))        # 256 CUs
            rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(h), 8, mask)
        assert rc == 0, rc
        out.append(h.value)
    return out


def part3():
    """Frames in flight over K streams of each kind: c2 full frames (the bench's pattern) and c4 rank band sets at
    N = 8 (band height 8), one context per stream slot."""
    kinds = os.environ.get("KINDS", "torch,hip,cumask").split(",")
    c2 = scenes.CONFIGS["c2"]
    for kind in kinds:
        for k in (1, 2, 3, 4):
            if kind == "torch":
                ts = [torch.cuda.Stream() for _ in range(k)]
                handles = [s.cuda_stream for s in ts]
            else:
                handles = make_streams(kind, k)
            for wl in ("c2", "c4r3"):
                if wl == "c2":
                    Wc, Hc, Bc, cm, sc, rows = c2.width, c2.height, c2.depth, c2.camera(), c2.scene(), None
                    npx = Hc
                else:
                    Wc, Hc, Bc, cm, sc = W, H, B, cam, cfg.scene()
                    rows = abi.rt_rows(8, 8, 3, 1)
                    npx = 272
                trs = [Tracer(0) for _ in range(k)]
                outs = []
                for tt in trs:
                    tt.set_scene(sc)
                    if wl == "c2":                       # the bench's outputs: RGBA32F + RGBA8
                        outs.append((torch.empty((npx, Wc, 4), dtype=torch.float32, device="cuda"),
                                     torch.empty((npx, Wc, 4), dtype=torch.uint8, device="cuda")))
                    else:
                        outs.append((None, torch.empty((npx, Wc), dtype=torch.uint8, device="cuda")))
                fmt = (abi.RT_PIXEL_RGBA32F, abi.RT_PIXEL_RGBA8) if wl == "c2" else (abi.RT_PIXEL_GRAY32F, abi.RT_PIXEL_GRAY8)
                la = [(trs[q]._ctx, ctypes.byref(cm), Wc, Hc, Bc, ctypes.byref(rows) if rows else None,
                       fmt[0], ctypes.c_void_p(outs[q][0].data_ptr()) if outs[q][0] is not None else None,
                       fmt[1], ctypes.c_void_p(outs[q][1].data_ptr()), ctypes.c_void_p(handles[q])) for q in range(k)]
                for a in la:
                    for _ in range(3):
                        abi.check(L.rt_render_dev_packed(*a), "first")
                torch.cuda.synchronize()
                cnt = [0]

                def f(la=la, cnt=cnt, k=k):
                    cnt[0] += 1
                    return L.rt_render_dev_packed(*la[cnt[0] % k])
                settle(f, 0.2)
                ms = statistics.median(wall_ms(f, 200, torch.cuda.synchronize) for _ in range(5))
                print(json.dumps({"part": 3, "stream_kind": kind, "streams": k, "workload": wl,
                                  "ms_per_frame": round(ms, 5)}), flush=True)
                for tt in trs:
                    tt.close()


def part4():
    """rank 0's unpack alone: an n-rank gathered GRAY8 (and RGB8) c4 buffer into the RGBA8 image."""
    st = torch.cuda.Stream()
    img = torch.empty((H, W, 4), dtype=torch.uint8, device="cuda")
    for n, hb_req in ((8, 8), (8, 0), (4, 0), (2, 0)):
        band, slab = ctypes.c_int(), ctypes.c_int()
        abi.check(L.rt_band_plan(H, n, hb_req, ctypes.byref(band), ctypes.byref(slab)), "rt_band_plan")
        hb, sr = band.value, slab.value
        out = {"part": 4, "n": n, "band_height": hb, "unpack_vec4_env": os.environ.get("RT_UNPACK_VEC4")}
        for fmt, ch in ((abi.RT_PIXEL_GRAY8, 1), (abi.RT_PIXEL_RGB8, 3)):
            gathered = torch.zeros((n * sr, W * ch), dtype=torch.uint8, device="cuda")
            up = lambda: L.rt_unpack_dev(ctypes.c_void_p(gathered.data_ptr()), ctypes.c_void_p(img.data_ptr()), W, H,  # noqa
                                         fmt, abi.RT_PIXEL_RGBA8, hb, n, sr, ctypes.c_void_p(st.cuda_stream))
            settle(up, 0.1)
            out["gray8_ms" if ch == 1 else "rgb8_ms"] = round(statistics.median(event_ms(up, 100, st) for _ in range(5)), 5)
        print(json.dumps(out), flush=True)


def part5():
    """Which hardware queues frames in flight land on (run under rocprofv3 --kernel-trace: Queue_Id per dispatch): for
    each stream kind, 3 streams taking 30 c2 frames in turn, kinds separated by 50 ms idle gaps; also prints each kind's
    per-frame interval over 200 frames."""
    c2 = scenes.CONFIGS["c2"]
    Wc, Hc, Bc, cm = c2.width, c2.height, c2.depth, c2.camera()
    for kind in os.environ.get("KINDS", "torch,hip,cumask,prio").split(","):
        if kind == "torch":
            handles = [torch.cuda.Stream().cuda_stream for _ in range(3)]
        elif kind == "prio":                                    # one stream per priority level
            handles = [torch.cuda.Stream(priority=p).cuda_stream for p in (0, -1, -2)]
        else:
            handles = make_streams(kind, 3)
        trs = [Tracer(0) for _ in range(3)]
        outs = []
        for tt in trs:
            tt.set_scene(c2.scene())
            outs.append((torch.empty((Hc, Wc, 4), dtype=torch.float32, device="cuda"),
                         torch.empty((Hc, Wc, 4), dtype=torch.uint8, device="cuda")))
        la = [(trs[q]._ctx, ctypes.byref(cm), Wc, Hc, Bc, None, ctypes.c_void_p(outs[q][0].data_ptr()),
               ctypes.c_void_p(outs[q][1].data_ptr()), None, None, ctypes.c_void_p(handles[q])) for q in range(3)]
        for a in la:
            for _ in range(3):
                abi.check(L.rt_render_dev(*a), "first")
        cnt = [0]

        def f(la=la, cnt=cnt):
            cnt[0] += 1
            return L.rt_render_dev(*la[cnt[0] % 3])
        settle(f, 0.1)
        time.sleep(0.05)
        ms = statistics.median(wall_ms(f, 200, torch.cuda.synchronize) for _ in range(3))
        time.sleep(0.05)
        print(json.dumps({"part": 5, "stream_kind": kind, "ms_per_frame": round(ms, 5)}), flush=True)
        for tt in trs:
            tt.close()


def part6():
    """Rank 0's pipeline at n = 8 (band height 8) as rt_render_multi runs it — its bands on two render streams in turn
    into NB frame buffers, each frame's unpack on the comm stream behind that frame's render, a buffer rendered into
    again once its unpack is done — for NB = 2, 3 and the comm stream at normal and high priority (r02-r05's group
    used the greatest), and the bands alone."""
    n = 8
    band, slab = ctypes.c_int(), ctypes.c_int()
    abi.check(L.rt_band_plan(H, n, 8, ctypes.byref(band), ctypes.byref(slab)), "rt_band_plan")
    hb, sr = band.value, slab.value
    img = torch.empty((H, W, 4), dtype=torch.uint8, device="cuda")
    for nb, prio, unpack in ((3, 0, True), (4, 0, True), (6, 0, True), (4, 0, "decoupled"), (4, 0, False)):
        t = Tracer(0)
        t.set_scene(cfg.scene())
        rows = abi.rt_rows(hb, n, 0, 1)
        sts = [torch.cuda.Stream() for _ in range(2)]
        cs = torch.cuda.Stream(priority=prio)
        gath = [torch.zeros((n * sr, W), dtype=torch.uint8, device="cuda") for _ in range(nb)]
        ev_r = [torch.cuda.Event() for _ in range(nb)]
        ev_a = [torch.cuda.Event() for _ in range(nb)]
        used = [False] * nb

        def frame(f, nb=nb, unpack=unpack, sts=sts, cs=cs, gath=gath, ev_r=ev_r, ev_a=ev_a, used=used, t=t, rows=rows):
            b, k = f % nb, f & 1
            if used[b] and unpack != "decoupled":          # decoupled: the root's bands go straight to the image
                sts[k].wait_event(ev_a[b])
            abi.check(L.rt_render_dev_packed(t._ctx, ctypes.byref(cam), W, H, B, ctypes.byref(rows), abi.RT_PIXEL_GRAY32F,
                                             None, abi.RT_PIXEL_GRAY8, ctypes.c_void_p(gath[b].data_ptr()),
                                             ctypes.c_void_p(sts[k].cuda_stream)), "render")
            ev_r[b].record(sts[k])
            if unpack:
                if unpack != "decoupled":
                    cs.wait_event(ev_r[b])
                abi.check(L.rt_unpack_dev(ctypes.c_void_p(gath[b].data_ptr()), ctypes.c_void_p(img.data_ptr()), W, H,
                                          abi.RT_PIXEL_GRAY8, abi.RT_PIXEL_RGBA8, hb, n, sr,
                                          ctypes.c_void_p(cs.cuda_stream)), "unpack")
            ev_a[b].record(cs if unpack else sts[k])
            used[b] = True
        for f in range(6):
            frame(f)
        torch.cuda.synchronize()
        cnt = [0]

        def g(frame=frame, cnt=cnt):
            cnt[0] += 1
            frame(cnt[0])
            return 0
        settle(g, 0.1)
        ms = [wall_ms(g, 120, torch.cuda.synchronize) for _ in range(3)]
        print(json.dumps({"part": 6, "buffers": nb, "comm_priority": prio, "unpack": unpack,
                          "ms_per_frame": [round(x, 5) for x in ms]}), flush=True)
        t.close()


if __name__ == "__main__":
    parts = os.environ.get("PARTS", "1,2").split(",")
    if "1" in parts:
        part1(int(os.environ.get("ROUNDS", "3")))
    if "2" in parts:
        part2([int(x) for x in os.environ.get("NS", "2,4,8").split(",")])
    if "3" in parts:
        part3()
    if "4" in parts:
        part4()
    if "5" in parts:
        part5()
    if "6" in parts:
        part6()
