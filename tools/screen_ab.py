#!/usr/bin/env python3
"""In-process interleaved A/B of rt_render_screen settings read from the environment at each call (RT_SCREEN_NEXT,
RT_SCREEN_NEXT_MIN, RT_SCREEN_AHEAD): one context, calls of the settings interleaved round by round, so process-
to-process differences (±5% on this host-bound path) cancel.  Every call's frame is compared with the first.
usage: SETTINGS='RT_SCREEN_NEXT=0;RT_SCREEN_NEXT_MIN=256' screen_ab.py [scene W H] [rounds]"""
import ctypes
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from ray_tracer_fragment_shader_amd import abi, scenes  # noqa: E402


def main():
    name, W, H = (sys.argv[1], int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else ("demo", 500, 500)
    rounds = int(sys.argv[4]) if len(sys.argv) > 4 else 9
    settings = [s for s in os.environ.get("SETTINGS", "RT_SCREEN_NEXT=0;RT_SCREEN_NEXT_MIN=0").split(";") if s]
    keys = {kv.split("=")[0] for s in settings for kv in s.split(",")}
    L = abi.lib()
    ctx = ctypes.c_void_p()
    abi.check(L.rt_ctx_create(0, ctypes.byref(ctx)), "rt_ctx_create")
    sa = scenes.CONFIGS[name].scene().to_abi()
    cam = scenes.make_camera(W, H, 1.0)
    rgb = np.zeros((H, W, 3), np.float64)
    ref = None
    res = {s: [] for s in settings}
    for r in range(rounds + 1):
        for s in settings:
            for k in keys:
                os.environ.pop(k, None)
            for kv in s.split(","):
                k, v = kv.split("=")
                os.environ[k] = v
            t = time.perf_counter()
            abi.check(L.rt_render_screen(ctx, ctypes.byref(sa), ctypes.byref(cam), W, H, 5, 0, 1, rgb.ctypes.data,
                                         None, None, None), "rt_render_screen")
            dt = time.perf_counter() - t
            if ref is None:
                ref = rgb.copy()
            assert np.array_equal(rgb, ref), s
            if r:
                res[s].append(dt)
    base = statistics.median(res[settings[0]])
    for s, v in res.items():
        print(json.dumps({"scene": name, "setting": s, "median_s": round(statistics.median(v), 4),
                          "min_s": round(min(v), 4), "vs_first": round(statistics.median(v) / base - 1, 4)}))
    L.rt_ctx_destroy(ctx)


if __name__ == "__main__":
    main()
