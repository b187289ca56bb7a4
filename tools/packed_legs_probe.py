#!/usr/bin/env python3
"""bench.py's draw() host-frame legs (packed_host_legs) in isolation: on a fresh context, after an rt_render RGBA8
call into torch-pinned memory (as in the bench), and with RT_COPY_KERNEL forced — where the pipelined frame's time goes."""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
from ray_tracer_fragment_shader_amd import abi, scenes  # noqa: E402
from ray_tracer_fragment_shader_amd.tracer import Tracer  # noqa: E402

L = abi.lib()
cfg = scenes.CONFIGS["c2"]
W, H, B = cfg.width, cfg.height, cfg.depth
sa, cam = cfg.scene().to_abi(), cfg.camera()
out = {}
t = Tracer(0)
out["fresh"] = bench.packed_host_legs(t, sa, cam, W, H, B)
out["fresh_again"] = bench.packed_host_legs(t, sa, cam, W, H, B)
t2 = Tracer(0)
host8 = torch.empty((H, W, 4), dtype=torch.uint8).pin_memory()
args_r = (t2._ctx, ctypes.byref(sa), ctypes.byref(cam), W, H, B, None, None, ctypes.c_void_p(host8.data_ptr()), None, None)
for _ in range(33):
    abi.check(L.rt_render(*args_r), "rt_render")
out["after_rt_render"] = bench.packed_host_legs(t2, sa, cam, W, H, B)
for k, v in out.items():
    print(k, json.dumps({a: b for a, b in v.items() if "ms" in a}), flush=True)
