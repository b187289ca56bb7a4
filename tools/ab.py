#!/usr/bin/env python3
"""Interleaved in-process timing of rt_render_dev across configs and kernel variants.

usage: ab.py c1,c2,c3,c5 MODE[,MODE...]   where MODE is a '+'-joined list of env settings applied when the
context is created, e.g. RT_SCENE_IN_LDS=1 or RT_MIN_WAVES=5+RT_SCENE_IN_LDS=0 ("base" = defaults).
Prints one JSON line per (config, mode) with median / min kernel ms."""
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


def main():
    cfgs = sys.argv[1].split(",") if len(sys.argv) > 1 else ["c1", "c2", "c3", "c5"]
    modes = sys.argv[2].split(",") if len(sys.argv) > 2 else ["base", "RT_SCENE_IN_LDS=1"]
    rounds = int(os.environ.get("ROUNDS", "5"))
    order = os.environ.get("TILE_ORDER")          # 0 adaptive / 1 bottom-to-top (rt_diag_tile_order)
    reps = int(os.environ.get("REPS", "20"))
    tracers = {}
    for m in modes:
        saved = dict(os.environ)
        if m != "base":
            for kv in m.split("+"):
                k, v = kv.split("=")
                os.environ[k] = v
        tracers[m] = Tracer(0)
        if order is not None and hasattr(abi.lib(), "rt_diag_tile_order"):
            abi.check(abi.lib().rt_diag_tile_order(tracers[m]._ctx, int(order)), "rt_diag_tile_order")
        os.environ.clear()
        os.environ.update(saved)
    res = {(c, m): [] for c in cfgs for m in modes}
    # untimed clock settle: back-to-back frames until the GPU clock reaches its loaded state
    cfg0 = scenes.CONFIGS[cfgs[0]]
    t0 = tracers[modes[0]]
    t0.set_scene(cfg0.scene())
    sb = t0.alloc(cfg0.width, cfg0.height, rgba32f=True, rgba8=True)
    end = time.perf_counter() + float(os.environ.get("SETTLE", "0.5"))
    while time.perf_counter() < end:
        for _ in range(16):
            t0.render_into(cfg0.camera(), cfg0.width, cfg0.height, cfg0.depth, sb)
        torch.cuda.synchronize()
    del sb
    bufs = {}
    for c in cfgs:
        cfg = scenes.CONFIGS[c]
        bufs[c] = tracers[modes[0]].alloc(cfg.width, cfg.height, rgba32f=True, rgba8=True)
    for _ in range(rounds):
        for c in cfgs:
            cfg = scenes.CONFIGS[c]
            cam = cfg.camera()
            for m in modes:
                t = tracers[m]
                t.set_scene(cfg.scene())
                t.render_into(cam, cfg.width, cfg.height, cfg.depth, bufs[c])   # warm
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                # pre-bound ctypes arguments: the host issues faster than the GPU drains (no host-bound gaps)
                fn = abi.lib().rt_render_dev
                la = (t._ctx, ctypes.byref(cam), cfg.width, cfg.height, cfg.depth, None,
                      ctypes.c_void_p(bufs[c]["rgba32f"].data_ptr()), ctypes.c_void_p(bufs[c]["rgba8"].data_ptr()),
                      None, None, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
                e0.record()
                for _ in range(reps):
                    fn(*la)
                e1.record()
                torch.cuda.synchronize()
                res[(c, m)].append(e0.elapsed_time(e1) / reps)
    for (c, m), v in res.items():
        rays = scenes.PINNED_RAYS[c]
        med = statistics.median(v)
        print(json.dumps({"config": c, "mode": m, "median_ms": round(med, 4), "min_ms": round(min(v), 4),
                          "Mray/s": round(rays / med / 1e3, 1)}))


if __name__ == "__main__":
    main()
