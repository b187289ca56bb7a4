#!/usr/bin/env python3
"""Back-to-back renders of one config's static view on one stream for SECONDS (default 3 s), for profilers that sample
the running kernel (rocprofv3 --pc-sampling).  usage: render_loop.py [config] [seconds]"""
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
    name = sys.argv[1] if len(sys.argv) > 1 else "c2"
    seconds = float(sys.argv[2]) if len(sys.argv) > 2 else 3.0
    L = abi.lib()
    cfg = scenes.CONFIGS[name]
    W, H, B = cfg.width, cfg.height, cfg.depth
    cam = cfg.camera()
    t = Tracer(0)
    t.set_scene(cfg.scene())
    st = torch.cuda.Stream()
    o32 = torch.empty((H, W, 4), dtype=torch.float32, device="cuda")
    o8 = torch.empty((H, W, 4), dtype=torch.uint8, device="cuda")
    args = (t._ctx, ctypes.byref(cam), W, H, B, None, ctypes.c_void_p(o32.data_ptr()), ctypes.c_void_p(o8.data_ptr()),
            None, None, ctypes.c_void_p(st.cuda_stream))
    n = 0
    t_end = time.perf_counter() + seconds
    while time.perf_counter() < t_end:
        for _ in range(32):
            abi.check(L.rt_render_dev(*args), "rt_render_dev")
        n += 32
        st.synchronize()
    print(f"{name}: {n} frames", flush=True)
    t.close()


if __name__ == "__main__":
    main()
