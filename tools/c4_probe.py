#!/usr/bin/env python3
"""Host vs device time of rt_render_multi on one GPU (a one-rank RCCL group, c3's frame): how long the host
takes to issue each call (no synchronisation) and the per-frame wall time with synchronisation."""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from ray_tracer_fragment_shader_amd import abi, scenes  # noqa: E402
from ray_tracer_fragment_shader_amd.tracer import Tracer  # noqa: E402


def main():
    L = abi.lib()
    cfg = scenes.CONFIGS["c3"]
    W, H, B = cfg.width, cfg.height, cfg.depth
    cam = cfg.camera()
    t = Tracer(0)
    t.set_scene(cfg.scene())
    g = ctypes.c_void_p()
    arr = (ctypes.c_void_p * 1)(t._ctx.value)
    abi.check(L.rt_group_create(arr, 1, abi.RT_TRANSPORT_RCCL, ctypes.byref(g)), "rt_group_create")
    img8 = torch.empty((H, W, 4), dtype=torch.uint8, device="cuda")
    st = torch.cuda.current_stream()
    argv = (g, ctypes.byref(cam), W, H, B, 0, abi.RT_OUT_RGBA8, None, ctypes.c_void_p(img8.data_ptr()),
            ctypes.c_void_p(st.cuda_stream))
    for _ in range(20):
        abi.check(L.rt_render_multi(*argv), "rt_render_multi")
    L.rt_group_synchronize(g)
    torch.cuda.synchronize()
    n = 40
    t0 = time.perf_counter()
    for _ in range(n):
        L.rt_render_multi(*argv)
    t1 = time.perf_counter()
    L.rt_group_synchronize(g)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"host issue {1e6 * (t1 - t0) / n:.1f} us/call, wall {1e6 * (t2 - t0) / n:.1f} us/frame")
    # plain renders of the same frame on one stream, for comparison
    bufs = t.alloc(W, H, rgba32f=False, rgba8=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        t.render_into(cam, W, H, B, bufs)
    torch.cuda.synchronize()
    print(f"rt_render_dev alone {1e6 * (time.perf_counter() - t0) / n:.1f} us/frame")
    L.rt_group_destroy(g)
    t.close()


if __name__ == "__main__":
    main()
