#!/usr/bin/env python3
"""Where does a frame's kernel time go?  Times rt_render_dev on pieces of one configuration:
full frame at depth 0..B, the bottom / top halves of the frame (same camera, shifted bottom_y), the
scene without spheres and without the board.  usage: split.py [config]   (prints one JSON line each)"""
import ctypes
import dataclasses
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from ray_tracer_fragment_shader_amd import abi, scenes  # noqa: E402
from ray_tracer_fragment_shader_amd.tracer import Tracer  # noqa: E402


def timed(t, cam, W, H, depth, bufs, reps=20, rounds=5):
    t.render_into(cam, W, H, depth, bufs)
    out = []
    for _ in range(rounds):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            t.render_into(cam, W, H, depth, bufs)
        e1.record()
        torch.cuda.synchronize()
        out.append(e0.elapsed_time(e1) / reps)
    return statistics.median(out)


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "c2"
    cfg = scenes.CONFIGS[name]
    W, H = cfg.width, cfg.height
    t = Tracer(0)
    bufs = t.alloc(W, H, rgba32f=True, rgba8=True)
    cam = cfg.camera()
    sc = cfg.scene()
    t.set_scene(sc)

    def rep(label, ms, **kw):
        print(json.dumps({"config": name, "piece": label, "ms": round(ms, 4), **kw}), flush=True)

    for d in range(cfg.depth + 1):
        rep(f"full depth {d}", timed(t, cam, W, H, d, bufs))
    half = H // 2
    for k, label in ((0, "bottom half"), (1, "top half")):
        c2 = abi.rt_camera()
        ctypes.pointer(c2)[0] = cam
        c2.bottom_y = cam.bottom_y + k * half
        rep(label, timed(t, c2, W, half, cfg.depth, bufs))
    for label, s in (("no spheres", dataclasses.replace(sc, spheres=[])),
                     ("no board", dataclasses.replace(sc, has_board=False)),
                     ("empty", dataclasses.replace(sc, spheres=[], has_board=False))):
        t.set_scene(s)
        for d in sorted({0, cfg.depth}):
            rep(f"{label} depth {d}", timed(t, cam, W, H, d, bufs))
    for label, kw in (("rgba8 only", dict(rgba32f=False, rgba8=True)),
                      ("rgba32f only", dict(rgba32f=True, rgba8=False))):
        b2 = t.alloc(W, H, **kw)
        for lab2, s in (("", sc), (" empty", dataclasses.replace(sc, spheres=[], has_board=False))):
            t.set_scene(s)
            rep(label + lab2, timed(t, cam, W, H, cfg.depth, b2))
    t.set_scene(sc)


if __name__ == "__main__":
    main()
