#!/usr/bin/env python3
"""bench.py's moving-camera leg (c2, 16-view orbit, a new eye every frame, 3 contexts on 3 streams) in a fresh process,
by stream set: three torch streams, the null stream + two torch streams, and three torch streams created after 24 other
streams (as in the bench, whose earlier legs create streams of their own).  Prints one JSON line per case."""
import ctypes
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from ray_tracer_fragment_shader_amd import abi, scenes  # noqa: E402
from ray_tracer_fragment_shader_amd.tracer import Tracer  # noqa: E402


def run(case, ts, ss, views, bufs, L, W, H, B, k=96):
    n = len(ts)
    la = [(ts[i % n]._ctx, ctypes.byref(views[i % 16]), W, H, B, None, ctypes.c_void_p(bufs[i % n][0].data_ptr()),
           ctypes.c_void_p(bufs[i % n][1].data_ptr()), None, None,
           ctypes.c_void_p(ss[i % n].cuda_stream if ss[i % n] is not None else 0)) for i in range(16 * n)]
    t_end = time.perf_counter() + 0.5                      # settle the clocks
    j = 0
    while time.perf_counter() < t_end:
        for _ in range(16):
            abi.check(L.rt_render_dev(*la[j % len(la)]), "rt_render_dev")
            j += 1
        torch.cuda.synchronize()
    best = None
    for _ in range(5):
        t0 = time.perf_counter()
        for i in range(k):
            abi.check(L.rt_render_dev(*la[i % len(la)]), "rt_render_dev")
        torch.cuda.synchronize()
        w = (time.perf_counter() - t0) / k * 1e3
        best = w if best is None else min(best, w)
    print(json.dumps({"case": case, "ms_per_frame": round(best, 4)}), flush=True)


def main():
    L = abi.lib()
    cfg = scenes.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "c2"]
    W, H, B = cfg.width, cfg.height, cfg.depth
    views = []
    for v in range(16):
        c = cfg.camera()
        ang = 2.0 * math.pi * v / 16
        c.eye = abi.vec3((60.0 * math.sin(ang), 100.0 + 10.0 * math.cos(ang), 200.0))
        views.append(c)
    ts = [Tracer(0) for _ in range(3)]
    for t in ts:
        t.set_scene(cfg.scene())
    bufs = [(torch.empty((H, W, 4), dtype=torch.float32, device="cuda"),
             torch.empty((H, W, 4), dtype=torch.uint8, device="cuda")) for _ in range(3)]
    run("three_torch_streams", ts, [torch.cuda.Stream() for _ in range(3)], views, bufs, L, W, H, B)
    run("null_plus_two", ts, [None, torch.cuda.Stream(), torch.cuda.Stream()], views, bufs, L, W, H, B)
    keep = [torch.cuda.Stream() for _ in range(24)]
    run("after_24_streams", ts, [torch.cuda.Stream() for _ in range(3)], views, bufs, L, W, H, B)
    run("one_stream_serial", ts[:1], [torch.cuda.Stream()], views, bufs, L, W, H, B)
    # the bench's first context has rendered the static view (calibrated: its tile-row order is the static view's)
    cam = cfg.camera()
    st = torch.cuda.Stream()
    for t in ts[:1]:
        for _ in range(4):
            abi.check(L.rt_render_dev(t._ctx, ctypes.byref(cam), W, H, B, None, ctypes.c_void_p(bufs[0][0].data_ptr()),
                                      ctypes.c_void_p(bufs[0][1].data_ptr()), None, None,
                                      ctypes.c_void_p(st.cuda_stream)), "rt_render_dev")
    torch.cuda.synchronize()
    run("first_ctx_calibrated_static", ts, [torch.cuda.Stream() for _ in range(3)], views, bufs, L, W, H, B)
    for t in ts:
        for _ in range(4):
            abi.check(L.rt_render_dev(t._ctx, ctypes.byref(cam), W, H, B, None, ctypes.c_void_p(bufs[0][0].data_ptr()),
                                      ctypes.c_void_p(bufs[0][1].data_ptr()), None, None,
                                      ctypes.c_void_p(st.cuda_stream)), "rt_render_dev")
    torch.cuda.synchronize()
    run("all_ctx_calibrated_static", ts, [torch.cuda.Stream() for _ in range(3)], views, bufs, L, W, H, B)
    fresh = [Tracer(0) for _ in range(3)]
    for t in fresh:
        t.set_scene(cfg.scene())
    run("fresh_again", fresh, [torch.cuda.Stream() for _ in range(3)], views, bufs, L, W, H, B)
    for t in fresh:
        t.close()
    # the same with the moving camera's re-timing off (RT_RECALIBRATE=0: the static view's order is kept) and at 32
    for rc in ("default", "0", "8"):                       # default: identity order; else RT_MOVING_ORDER=1
        if rc != "default":
            os.environ["RT_MOVING_ORDER"], os.environ["RT_RECALIBRATE"] = "1", rc
        cal = [Tracer(0) for _ in range(3)]
        for t in cal:
            t.set_scene(cfg.scene())
            for _ in range(4):
                abi.check(L.rt_render_dev(t._ctx, ctypes.byref(cam), W, H, B, None,
                                          ctypes.c_void_p(bufs[0][0].data_ptr()), ctypes.c_void_p(bufs[0][1].data_ptr()),
                                          None, None, ctypes.c_void_p(st.cuda_stream)), "rt_render_dev")
        torch.cuda.synchronize()
        run(f"all_calibrated_recalibrate_{rc}", cal, [torch.cuda.Stream() for _ in range(3)], views, bufs, L, W, H, B)
        for t in cal:
            t.close()
    os.environ.pop("RT_RECALIBRATE", None)
    os.environ.pop("RT_MOVING_ORDER", None)
    del keep
    for t in ts:
        t.close()


if __name__ == "__main__":
    main()
