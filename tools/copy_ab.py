#!/usr/bin/env python3
"""draw()'s host-frame path at c2 (GRAY8, pinned): A/B of where the device-to-host copy runs.

Settings (env read at rt_ctx_create; SETTINGS=mode:blocks[:split[:chunks[:writer]]]): RT_COPY_MODE 1 = copy kernel on the render stream (serial), 0 = copy kernel
on the context's copy stream (overlaps the next render), 2 = the render kernel stores straight into the pinned
host buffer (no copy), 3 = an SDMA engine copies it (HSA, no CUs); RT_COPY_BLOCKS = copy-kernel workgroups (0 = auto,
up to 1024).  Every setting's frames are
checked byte for byte against a device render; rounds interleave the settings (one process, one GPU)."""
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

# mode:blocks[:split[:chunks]] — RT_SDMA_SPLIT (engines an SDMA frame copy is split over); RT_SDMA_CHUNKS (row chunks
# of a synchronous SDMA frame) was an r05 experiment, no longer read; writer = RT_SDMA_WRITER (how the render stream
# starts the SDMA copy: 1 stream write-value, 2 signal kernel, 0 the library's choice)
_DEFAULTS = ["1", "0", "2", "2", "0"]                      # (mode, blocks, split, chunks, writer)
SETTINGS = [tuple(x.split(":") + _DEFAULTS[len(x.split(":")):]) for x in
            os.environ.get("SETTINGS", "1:0,0:0,0:64,0:16,1:64,2:0").split(",")]
# (RT_COPY_KERNEL=0 in the environment: hipMemcpyAsync — the runtime's blit kernel — instead of the copy kernel)
L = abi.lib()
cfg = scenes.CONFIGS["c2"]
W, H, B = cfg.width, cfg.height, cfg.depth
sa, cam = cfg.scene().to_abi(), cfg.camera()
ref = Tracer(0)
ref.set_scene(cfg.scene())
_, want = ref.render_packed(cam, W, H, B, byte_format=abi.RT_PIXEL_GRAY8)
torch.cuda.synchronize()
want = want.cpu().numpy().reshape(-1)
ctxs = {}
for mode, blocks, split, chunks, writer in SETTINGS:
    os.environ["RT_COPY_MODE"], os.environ["RT_COPY_BLOCKS"] = mode, blocks
    os.environ["RT_SDMA_SPLIT"], os.environ["RT_SDMA_CHUNKS"] = split, chunks
    os.environ["RT_SDMA_WRITER"] = writer
    ctxs[(mode, blocks, split, chunks, writer)] = Tracer(0)
pins = []
for _ in range(3):
    p = ctypes.c_void_p()
    abi.check(L.rt_host_alloc(W * H, ctypes.byref(p)), "rt_host_alloc")
    pins.append(p)
res = {k: {"sync": [], "pipe1": [], "pipe2": []} for k in ctxs}
k = 60
fmt = abi.RT_PIXEL_GRAY8
for rnd in range(int(os.environ.get("ROUNDS", "5"))):
    for key, t in ctxs.items():
        a = (t._ctx, ctypes.byref(sa), ctypes.byref(cam), W, H, B, fmt)
        for _ in range(4):
            abi.check(L.rt_render_packed(*a, pins[0], None), "sync")
        got = (ctypes.c_uint8 * (W * H)).from_address(pins[0].value)
        import numpy as np
        assert np.array_equal(np.frombuffer(got, np.uint8), want), f"{key}: frame differs"
        t0 = time.perf_counter()
        for _ in range(k):
            L.rt_render_packed(*a, pins[0], None)
        res[key]["sync"].append((time.perf_counter() - t0) / k * 1e6)
        for depth in (1, 2):
            tk = [ctypes.c_uint64() for _ in range(3)]
            abi.check(L.rt_ctx_wait(t._ctx, 0), "wait")
            t0 = time.perf_counter()
            for f in range(k):
                abi.check(L.rt_render_packed_async(*a, pins[f % 3], ctypes.byref(tk[f % 3])), "async")
                if f >= depth:
                    abi.check(L.rt_ctx_wait(t._ctx, tk[(f - depth) % 3].value), "wait")
            abi.check(L.rt_ctx_wait(t._ctx, 0), "wait")
            res[key][f"pipe{depth}"].append((time.perf_counter() - t0) / k * 1e6)
            for j in range(3):
                got = (ctypes.c_uint8 * (W * H)).from_address(pins[j].value)
                assert np.array_equal(np.frombuffer(got, np.uint8), want), f"{key}: pipelined frame differs"
out = {f"mode{m}_blocks{b}" + (f"_split{sp}_writer{w}" if m == "3" else ""):
       {n: round(statistics.median(v), 1) for n, v in d.items()} for (m, b, sp, ch, w), d in res.items()}
print(json.dumps({"us_per_frame_median": out, "frames": k}, indent=1))
for p in pins:
    L.rt_host_free(p)
