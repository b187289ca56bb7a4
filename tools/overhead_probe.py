#!/usr/bin/env python3
"""Fixed costs of a short timed region at c2 (bench.py's 20-step driver run): per-frame GPU interval (HIP events
around the launches, 3 streams) against host wall time for K frames, with the region ended by
torch.cuda.synchronize() alone or by spinning on the last frame's event first; plus the host cost of one
rt_render_dev call and the launch-to-start latency of the first frame."""
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
cfg = scenes.CONFIGS["c2"]
W, H, B = cfg.width, cfg.height, cfg.depth
cam = cfg.camera()
nf = 3
trs = [Tracer(0) for _ in range(nf)]
for t in trs:
    t.set_scene(cfg.scene())
sts = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(nf - 1)]
outs = [(torch.empty((H, W, 4), dtype=torch.float32, device="cuda"), torch.empty((H, W, 4), dtype=torch.uint8,
                                                                                  device="cuda")) for _ in range(nf)]
la = [(trs[i]._ctx, ctypes.byref(cam), W, H, B, None, ctypes.c_void_p(outs[i][0].data_ptr()),
       ctypes.c_void_p(outs[i][1].data_ptr()), None, None, ctypes.c_void_p(sts[i].cuda_stream)) for i in range(nf)]
fn = L.rt_render_dev
for _ in range(30):
    for a in la:
        fn(*a)
torch.cuda.synchronize()
res = {"sync": [], "spin": [], "nowait": [], "interval": [], "interval_nowait": [], "host_call_us": []}
K = int(os.environ.get("K", "20"))
for rnd in range(15):
    t_end = time.perf_counter() + 0.1
    while time.perf_counter() < t_end:
        for a in la:
            fn(*a)
        torch.cuda.synchronize()
    for mode in ("sync", "spin"):
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        last = torch.cuda.Event()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ev0.record(sts[0])
        for s in sts[1:]:
            s.wait_event(ev0)
        t_call = time.perf_counter()
        for i in range(K):
            fn(*la[i % nf])
            if i == 0:
                t_call = time.perf_counter() - t_call
        for s in sts[1:]:
            e = torch.cuda.Event()
            e.record(s)
            sts[0].wait_event(e)
        ev1.record(sts[0])
        if mode == "spin":
            while not ev1.query():
                pass
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        res[mode].append(wall / K * 1e6)
        res["interval"].append(ev0.elapsed_time(ev1) / K * 1e3)
        res["host_call_us"].append(t_call * 1e6)
    # bench.py r04: no cross-stream waits in the region, an end stamp per stream
    ev0 = torch.cuda.Event(enable_timing=True)
    ends = [torch.cuda.Event(enable_timing=True) for _ in sts]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record(sts[0])
    for i in range(K):
        fn(*la[i % nf])
    for e, s in zip(ends, sts):
        e.record(s)
    torch.cuda.synchronize()
    res["nowait"].append((time.perf_counter() - t0) / K * 1e6)
    res["interval_nowait"].append(max(ev0.elapsed_time(e) for e in ends) / K * 1e3)
print(json.dumps({k: round(statistics.median(v), 2) for k, v in res.items() if v} | {"K": K}))
