#!/usr/bin/env python3
"""Host-side cost per rt_render_dev launch (c1 frame, ~9 us kernel) for several call styles."""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from ray_tracer_fragment_shader_amd import abi, scenes  # noqa: E402
from ray_tracer_fragment_shader_amd.tracer import Tracer  # noqa: E402

cfg = scenes.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "c1"]
tr = Tracer(0)
tr.set_scene(cfg.scene())
cam = cfg.camera()
bufs = tr.alloc(cfg.width, cfg.height, rgba32f=True, rgba8=True)
st = torch.cuda.current_stream()
L = abi.lib()
args = (tr._ctx, ctypes.byref(cam), cfg.width, cfg.height, cfg.depth, None,
        ctypes.c_void_p(bufs["rgba32f"].data_ptr()), ctypes.c_void_p(bufs["rgba8"].data_ptr()), None, None,
        ctypes.c_void_p(st.cuda_stream))
fn = L.rt_render_dev
hip = ctypes.CDLL("libamdhip64.so")
N = 400
evs = [ctypes.c_void_p() for _ in range(2 * N)]
for e in evs:
    hip.hipEventCreate(ctypes.byref(e))
tev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * N)]


def run(name, body):
    torch.cuda.synchronize()
    t = time.perf_counter()
    for k in range(N):
        body(k)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / N * 1e6
    print(f"{name:40s} {dt:8.2f} us/launch")


for _ in range(2):
    run("Tracer.render_into", lambda k: tr.render_into(cam, cfg.width, cfg.height, cfg.depth, bufs))
    run("prebound fn(*args)", lambda k: fn(*args))
    run("prebound + torch events", lambda k: (tev[2 * k].record(st), fn(*args), tev[2 * k + 1].record(st)))
    run("prebound + hipEventRecord", lambda k: (hip.hipEventRecord(evs[2 * k], args[-1]), fn(*args),
                                                hip.hipEventRecord(evs[2 * k + 1], args[-1])))
ms = ctypes.c_float()
hip.hipEventElapsedTime(ctypes.byref(ms), evs[0], evs[1])
print("kernel (hip events) us", ms.value * 1e3)
