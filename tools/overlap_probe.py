#!/usr/bin/env python3
"""Per-frame throughput of back-to-back independent c2 frames on 1, 2, 3 or 4 HIP streams (one context and
one set of output buffers per stream; frames round-robin over the streams).  Measures how much of a launch's
ramp-up and tail the next frame's launch can fill.  usage: overlap_probe.py [config] [frames]"""
import ctypes
import sys
import time

import torch

sys.path.insert(0, ".")
from ray_tracer_fragment_shader_amd import abi, scenes  # noqa: E402
from ray_tracer_fragment_shader_amd.tracer import Tracer  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "c2"
K = int(sys.argv[2]) if len(sys.argv) > 2 else 200
cfg = scenes.CONFIGS[name]
W, H, B = cfg.width, cfg.height, cfg.depth
cam = cfg.camera()
L = abi.lib()
res = {}
for ns in (1, 2, 3, 4, 1, 2):
    trs = [Tracer(0) for _ in range(ns)]
    for t in trs:
        t.set_scene(cfg.scene())
    streams = [torch.cuda.Stream() for _ in range(ns)]
    bufs = [t.alloc(W, H, rgba32f=True, rgba8=True) for t in trs]
    args = [(trs[i]._ctx, ctypes.byref(cam), W, H, B, None, ctypes.c_void_p(bufs[i]["rgba32f"].data_ptr()),
             ctypes.c_void_p(bufs[i]["rgba8"].data_ptr()), None, None, ctypes.c_void_p(streams[i].cuda_stream))
            for i in range(ns)]
    for _ in range(4):
        for a in args:
            abi.check(L.rt_render_dev(*a), "rt_render_dev")
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s0 = streams[0]
    e0.record(s0)
    for s in streams[1:]:
        s.wait_event(e0)
    t0 = time.perf_counter()
    for k in range(K):
        L.rt_render_dev(*args[k % ns])
    ends = []
    for s in streams[1:]:
        ev = torch.cuda.Event()
        ev.record(s)
        s0.wait_event(ev)
    e1.record(s0)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / K * 1e6
    res.setdefault(ns, []).append((round(e0.elapsed_time(e1) / K * 1e3, 2), round(wall, 2)))
    for t in trs:
        t.close()
print(name, "us per frame (events, wall) by streams:", res)
