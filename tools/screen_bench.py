#!/usr/bin/env python3
"""Time the reference-faithful rayTraceScreen: rt_render_screen (GPU chunks) vs the serial C restatement
(oracle/rt_oracle.c, one core — the frame is a serial chain).  RT_SCREEN_PROFILE=1 prints the phases.
usage: screen_bench.py [scene W H ...]        LIB=<path>: another build of librt_amd.so (A/B)"""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from oracle import pyoracle as po  # noqa: E402
from ray_tracer_fragment_shader_amd import abi, scenes  # noqa: E402


def load_lib():
    path = os.environ.get("LIB")
    if not path:
        return abi.lib()
    L = ctypes.CDLL(path)
    for fn, (res, argt) in abi.SIGNATURES.items():
        if hasattr(L, fn):
            getattr(L, fn).restype = res
            getattr(L, fn).argtypes = argt
    return L


def main():
    args = sys.argv[1:] or ["demo", "500", "500", "c2", "640", "360"]
    L = load_lib()
    ctx = ctypes.c_void_p()
    abi.check(L.rt_ctx_create(0, ctypes.byref(ctx)), "rt_ctx_create")
    for k in range(0, len(args), 3):
        name, W, H = args[k], int(args[k + 1]), int(args[k + 2])
        sc = scenes.CONFIGS[name].scene()
        sa = sc.to_abi()
        cam = scenes.make_camera(W, H, 1.0)
        rgb = np.zeros((H, W, 3), np.float64)
        ns = np.zeros((H, W), np.uint8)
        calls = ctypes.c_uint64()
        # warm-up call (first launch of the trace kernel variant, host/device allocations), then timed
        abi.check(L.rt_render_screen(ctx, ctypes.byref(sa), ctypes.byref(cam), W, H, 5, 0, 1,
                                             rgb.ctypes.data, None, ns.ctypes.data, ctypes.byref(calls)),
                  "rt_render_screen")
        times = []
        for _ in range(int(os.environ.get("REPS", "5"))):    # (the frame is host-bound: the median of a few calls)
            t = time.perf_counter()
            abi.check(L.rt_render_screen(ctx, ctypes.byref(sa), ctypes.byref(cam), W, H, 5, 0, 1,
                                         rgb.ctypes.data, None, ns.ctypes.data, ctypes.byref(calls)),
                      "rt_render_screen")
            times.append(time.perf_counter() - t)
        times.sort()
        t_gpu = times[len(times) // 2]
        t = time.perf_counter()
        want, want_ns, want_calls = po.render_screen(sa, W, H, 5, po.GLIBC, 1)
        t_cpu = time.perf_counter() - t
        print(json.dumps({"scene": name, "width": W, "height": H, "samples": int(ns.sum()),
                          "gpu_s": round(t_gpu, 4), "gpu_s_min": round(times[0], 4), "cpu_serial_s": round(t_cpu, 3),
                          "speedup": round(t_cpu / t_gpu, 2),
                          "bit_exact": bool(np.array_equal(rgb, want) and calls.value == want_calls)}), flush=True)


if __name__ == "__main__":
    main()
