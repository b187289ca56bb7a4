#!/usr/bin/env python3
"""rt_render (synchronous, RGBA8 into torch pin_memory()) at c2: the product's copy kernel vs hipMemcpyAsync
(RT_COPY_KERNEL=0 at context creation), two contexts in one process, calls interleaved; frames compared."""
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
sa, cam = cfg.scene().to_abi(), cfg.camera()
ctxs = {}
for name, v in (("copy_kernel", "-1"), ("memcpy", "0")):
    os.environ["RT_COPY_KERNEL"] = v
    ctxs[name] = Tracer(0)
os.environ.pop("RT_COPY_KERNEL")
outs = {n: torch.empty((H, W, 4), dtype=torch.uint8).pin_memory() for n in ctxs}
res = {n: [] for n in ctxs}
for r in range(int(os.environ.get("ROUNDS", "7")) + 1):
    for n, t in ctxs.items():
        args = (t._ctx, ctypes.byref(sa), ctypes.byref(cam), W, H, B, None, None,
                ctypes.c_void_p(outs[n].data_ptr()), None, None)
        for _ in range(3):
            abi.check(L.rt_render(*args), "rt_render")
        t0 = time.perf_counter()
        for _ in range(20):
            L.rt_render(*args)
        if r:
            res[n].append((time.perf_counter() - t0) / 20 * 1e3)
assert torch.equal(outs["copy_kernel"], outs["memcpy"])
for n, v in res.items():
    print(json.dumps({"rt_render_rgba8": n, "median_ms": round(statistics.median(v), 4), "min_ms": round(min(v), 4)}))
