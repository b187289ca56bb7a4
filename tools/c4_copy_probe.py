#!/usr/bin/env python3
"""rt_render_multi on one GPU with n COPY-transport ranks (c3's 3840x2160 frame, GRAY8 wire): per-phase times
from rt_group_get_stats and the per-frame wall time, for each setting of an A/B environment variable (AB_VAR, default
RT_GROUP_COMM_PRIORITY: the comm streams at the default or the greatest priority; RT_GATHER_ROOT_WAITS: the root's
gather posted at once or after its own render).  Frames are checked byte for byte against a one-launch render."""
import ctypes
import json
import os
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
sc = cfg.scene()
one = Tracer(0)
one.set_scene(sc)
want = one.render(cam, W, H, B, rgba32f=False, rgba8=True)["rgba8"]
torch.cuda.synchronize()
out = {}
for rnd in range(int(os.environ.get("ROUNDS", "3"))):
    for n in (2, 4, 8):
        for waits in os.environ.get("AB_VALUES", "0,1").split(","):
            os.environ[os.environ.get("AB_VAR", "RT_GROUP_COMM_PRIORITY")] = waits
            ctxs = [Tracer(0) for _ in range(n)]
            for c in ctxs:
                c.set_scene(sc)
            arr = (ctypes.c_void_p * n)(*[c._ctx.value for c in ctxs])
            g = ctypes.c_void_p()
            abi.check(L.rt_group_create(arr, n, abi.RT_TRANSPORT_COPY, ctypes.byref(g)), "rt_group_create")
            img = torch.empty((H, W, 4), dtype=torch.uint8, device="cuda")
            st = torch.cuda.Stream()
            argv = (g, ctypes.byref(cam), W, H, B, 0, abi.RT_OUT_RGBA8, None, ctypes.c_void_p(img.data_ptr()),
                    ctypes.c_void_p(st.cuda_stream))
            for _ in range(12):
                abi.check(L.rt_render_multi(*argv), "rt_render_multi")
            abi.check(L.rt_group_synchronize(g), "sync")
            torch.cuda.synchronize()
            assert torch.equal(img, want), (n, waits)
            k = 30
            t0 = time.perf_counter()
            for _ in range(k):
                abi.check(L.rt_render_multi(*argv), "rt_render_multi")
            abi.check(L.rt_group_synchronize(g), "sync")
            torch.cuda.synchronize()
            wall = (time.perf_counter() - t0) / k * 1e3
            abi.check(L.rt_group_timing(g, 1), "timing")
            for _ in range(k):
                abi.check(L.rt_render_multi(*argv), "rt_render_multi")
            s = abi.rt_group_stats()
            abi.check(L.rt_group_get_stats(g, ctypes.byref(s)), "stats")
            torch.cuda.synchronize()
            assert torch.equal(img, want), (n, waits)
            key = f"n{n}_{os.environ.get('AB_VAR', 'RT_GROUP_COMM_PRIORITY')}={waits}"
            out.setdefault(key, []).append({"wall_ms": round(wall, 4), "render_ms": round(s.render_ms, 4),
                                            "gather_ms": round(s.gather_ms, 4), "assemble_ms": round(s.assemble_ms, 4),
                                            "frame_ms": round(s.frame_ms, 4)})
            L.rt_group_destroy(g)
            for c in ctxs:
                c.close()
print(json.dumps(out, indent=1))
