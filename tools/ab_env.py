#!/usr/bin/env python3
"""In-process, interleaved A/B of context settings read from the environment at rt_ctx_create (RT_PERSIST,
RT_PERSIST_WAVES, RT_CONE_CACHE, ...): one context per mode in ONE process, renders interleaved round by round
(box and process clock differences cancel out), every mode's RGBA32F + RGBA8 frame compared byte for byte with
the first mode's.

usage: ab_env.py c2,c3,c5 rounds 'base:' 'persist:RT_PERSIST=1' 'p7:RT_PERSIST=1,RT_PERSIST_WAVES=7' ...
prints one JSON line per (config, mode): median / min kernel ms, vs the first mode, frames identical
"""
import ctypes
import json
import math
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from ray_tracer_fragment_shader_amd import abi, scenes  # noqa: E402


def main():
    cfgs = sys.argv[1].split(",")
    rounds = int(sys.argv[2])
    modes = []
    for spec in sys.argv[3:]:
        name, _, kv = spec.partition(":")
        env = dict(p.split("=", 1) for p in kv.split(",") if p)
        modes.append((name, env))
    reps = int(os.environ.get("REPS", "20"))
    moving = os.environ.get("MOVING", "0") == "1"      # a new eye every render (16-view orbit, as bench.py's leg)
    L = abi.lib()
    ctxs = {}
    for name, env in modes:
        saved = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        c = ctypes.c_void_p()
        abi.check(L.rt_ctx_create(0, ctypes.byref(c)), "rt_ctx_create")
        ctxs[name] = c
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    st = torch.cuda.current_stream()
    res = {(c, n): [] for c in cfgs for n, _ in modes}
    same = {(c, n): True for c in cfgs for n, _ in modes}
    bufs = {}
    for c in cfgs:
        cfg = scenes.CONFIGS[c]
        bufs[c] = {n: (torch.empty((cfg.height, cfg.width, 4), dtype=torch.float32, device="cuda"),
                       torch.empty((cfg.height, cfg.width, 4), dtype=torch.uint8, device="cuda")) for n, _ in modes}
    for r in range(rounds + 1):                       # round 0: untimed warm-up / calibration / clock settle
        for c in cfgs:
            cfg = scenes.CONFIGS[c]
            sa = cfg.scene().to_abi()
            cams = [cfg.camera()]
            if moving:
                cams = []
                for v in range(16):
                    cm = cfg.camera()
                    ang = 2.0 * 3.141592653589793 * v / 16
                    cm.eye = abi.vec3((60.0 * math.sin(ang), 100.0 + 10.0 * math.cos(ang), 200.0))
                    cams.append(cm)
            for name, _ in modes:
                b32, b8 = bufs[c][name]
                abi.check(L.rt_set_scene(ctxs[name], ctypes.byref(sa)), "rt_set_scene")
                las = [(ctxs[name], ctypes.byref(cam), cfg.width, cfg.height, cfg.depth, None,
                        ctypes.c_void_p(b32.data_ptr()), ctypes.c_void_p(b8.data_ptr()), None, None,
                        ctypes.c_void_p(st.cuda_stream)) for cam in cams]
                for i in range(3 if r else 40):
                    abi.check(L.rt_render_dev(*las[i % len(las)]), "rt_render_dev")
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record()
                for i in range(reps):
                    L.rt_render_dev(*las[i % len(las)])
                e1.record()
                torch.cuda.synchronize()
                if r:
                    res[(c, name)].append(e0.elapsed_time(e1) / reps)
                else:
                    ref32, ref8 = bufs[c][modes[0][0]]
                    same[(c, name)] = bool(torch.equal(b32, ref32) and torch.equal(b8, ref8))
    first = modes[0][0]
    for (c, name), v in res.items():
        base = statistics.median(res[(c, first)])
        med = statistics.median(v)
        print(json.dumps({"config": c, "mode": name, "median_ms": round(med, 4), "min_ms": round(min(v), 4),
                          "vs_first": round(med / base - 1, 4), "identical": same[(c, name)]}), flush=True)
    for name, _ in modes:
        L.rt_ctx_destroy(ctxs[name])


if __name__ == "__main__":
    main()
