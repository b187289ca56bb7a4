#!/usr/bin/env python3
"""Host-frame timing probe (rt_render_packed / rt_render_packed_async) at c2: where draw()'s time goes."""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

from ray_tracer_fragment_shader_amd import abi, scenes  # noqa: E402
from ray_tracer_fragment_shader_amd.tracer import Tracer  # noqa: E402

L = abi.lib()
cfg = scenes.CONFIGS["c2"]
W, H, B = cfg.width, cfg.height, cfg.depth
sa, cam = cfg.scene().to_abi(), cfg.camera()
t = Tracer(0)
pins = []
for _ in range(2):
    p = ctypes.c_void_p()
    abi.check(L.rt_host_alloc(W * H * 4, ctypes.byref(p)), "rt_host_alloc")
    pins.append(p)
for fmt, name in ((abi.RT_PIXEL_GRAY8, "gray8"), (abi.RT_PIXEL_RGBA8, "rgba8")):
    a = (t._ctx, ctypes.byref(sa), ctypes.byref(cam), W, H, B, fmt)
    for _ in range(5):
        abi.check(L.rt_render_packed(*a, pins[0], None), "sync")
    k = 50
    t0 = time.perf_counter()
    for _ in range(k):
        L.rt_render_packed(*a, pins[0], None)
    sync = (time.perf_counter() - t0) / k * 1e3
    tk = [ctypes.c_uint64(), ctypes.c_uint64()]
    abi.check(L.rt_ctx_wait(t._ctx, 0), "wait")
    t0 = time.perf_counter()
    for f in range(k):
        L.rt_render_packed_async(*a, pins[f & 1], ctypes.byref(tk[f & 1]))
        if f:
            L.rt_ctx_wait(t._ctx, tk[(f - 1) & 1].value)
    L.rt_ctx_wait(t._ctx, 0)
    pipe = (time.perf_counter() - t0) / k * 1e3
    t0 = time.perf_counter()
    for f in range(k):
        L.rt_render_packed_async(*a, pins[f & 1], ctypes.byref(tk[f & 1]))
    L.rt_ctx_wait(t._ctx, 0)
    queued = (time.perf_counter() - t0) / k * 1e3
    t0 = time.perf_counter()
    for f in range(k):
        L.rt_render_packed_async(*a, pins[f & 1], ctypes.byref(tk[f & 1]))
        L.rt_ctx_wait(t._ctx, tk[f & 1].value)
    each = (time.perf_counter() - t0) / k * 1e3
    print(f"{name}: sync {sync:.4f} ms/call, pipelined {pipe:.4f}, all-queued {queued:.4f}, "
          f"async+wait-each {each:.4f} ms/frame", flush=True)
for p in pins:
    L.rt_host_free(p)
t.close()
