#!/usr/bin/env python3
"""In-process, interleaved A/B of library builds: the in-tree lib/librt_amd.so ("base") and every
tools/_ab/<name>/librt_amd.so (r06: the experiment builds that travel to the GPU box; tools/_var stays local), each loaded as its own handle (copied to a private path) in ONE process, with
their renders interleaved round by round — so box-to-box and process-to-process clock differences (±2% at c2)
cancel out.

usage: ab_libs.py [c2,c3,c5] [rounds]        prints one JSON line per (config, lib): median / min kernel ms
INFLIGHT=k: bench.py's timed pattern instead — k contexts, streams and output buffers per build, frames issued
round-robin, per-frame interval = (last stream's end - start) / frames.
"""
import ctypes
import glob
import json
import math
import os
import shutil
import statistics
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from ray_tracer_fragment_shader_amd import abi, scenes  # noqa: E402


def load(path, tmp, name):
    dst = os.path.join(tmp, f"librt_{name}.so")
    shutil.copy(path, dst)
    L = ctypes.CDLL(dst)
    for fn, (res, args) in abi.SIGNATURES.items():
        if hasattr(L, fn):
            getattr(L, fn).restype = res
            getattr(L, fn).argtypes = args
    return L


def main():
    cfgs = sys.argv[1].split(",") if len(sys.argv) > 1 else ["c2", "c3", "c5"]
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 9
    reps = int(os.environ.get("REPS", "20"))
    moving = os.environ.get("MOVING", "0") == "1"      # a new eye every render (16-view orbit, as bench.py's leg)
    tmp = tempfile.mkdtemp()
    libs = {"base": load(abi.LIB_PATH, tmp, "base")}
    only = set(os.environ["VARS"].split(",")) if os.environ.get("VARS") else None
    for d in sorted(glob.glob(os.path.join(ROOT, "tools", os.environ.get("AB_DIR", "_ab"), "*", "librt_amd.so"))):
        name = os.path.basename(os.path.dirname(d))
        if only is None or name in only:
            libs[name] = load(d, tmp, name)
    st = torch.cuda.current_stream()
    nfly = int(os.environ.get("INFLIGHT", "0"))
    ctxs, bufs = {}, {}
    for name, L in libs.items():
        c = ctypes.c_void_p()
        abi.check(L.rt_ctx_create(0, ctypes.byref(c)), "rt_ctx_create")
        ctxs[name] = c
    fly_ctx = {}
    sts = [torch.cuda.Stream() for _ in range(nfly)]
    for name, L in libs.items():
        fly_ctx[name] = []
        for _ in range(nfly):
            c = ctypes.c_void_p()
            abi.check(L.rt_ctx_create(0, ctypes.byref(c)), "rt_ctx_create")
            fly_ctx[name].append(c)
    res = {(c, n): [] for c in cfgs for n in libs}
    fly_bufs = {}
    for c in cfgs:
        cfg = scenes.CONFIGS[c]
        bufs[c] = (torch.empty((cfg.height, cfg.width, 4), dtype=torch.float32, device="cuda"),
                   torch.empty((cfg.height, cfg.width, 4), dtype=torch.uint8, device="cuda"))
        fly_bufs[c] = [(torch.empty((cfg.height, cfg.width, 4), dtype=torch.float32, device="cuda"),
                        torch.empty((cfg.height, cfg.width, 4), dtype=torch.uint8, device="cuda"))
                       for _ in range(nfly)]
    for r in range(rounds + 1):                       # round 0: untimed warm-up / calibration / clock settle
        for c in cfgs:
            cfg = scenes.CONFIGS[c]
            sa = cfg.scene().to_abi()
            cams = [cfg.camera()]
            if moving:
                cams = []
                for v in range(16):
                    cm = cfg.camera()
                    ang = 2.0 * math.pi * v / 16
                    cm.eye = abi.vec3((60.0 * math.sin(ang), 100.0 + 10.0 * math.cos(ang), 200.0))
                    cams.append(cm)
            b32, b8 = bufs[c]
            for name, L in libs.items():
                if nfly:
                    fl = []
                    for j in range(nfly):
                        abi.check(L.rt_set_scene(fly_ctx[name][j], ctypes.byref(sa)), "rt_set_scene")
                        fl.append((fly_ctx[name][j], ctypes.byref(cams[0]), cfg.width, cfg.height, cfg.depth, None,
                                   ctypes.c_void_p(fly_bufs[c][j][0].data_ptr()),
                                   ctypes.c_void_p(fly_bufs[c][j][1].data_ptr()), None, None,
                                   ctypes.c_void_p(sts[j].cuda_stream)))
                    for i in range(3 * nfly if r else 40):
                        abi.check(L.rt_render_dev(*fl[i % nfly]), "rt_render_dev")
                    torch.cuda.synchronize()
                    e0 = torch.cuda.Event(enable_timing=True)
                    e0.record(sts[0])
                    for i in range(reps):
                        L.rt_render_dev(*fl[i % nfly])
                    ends = []
                    for j in range(nfly):
                        e = torch.cuda.Event(enable_timing=True)
                        e.record(sts[j])
                        ends.append(e)
                    torch.cuda.synchronize()
                    if r:
                        res[(c, name)].append(max(e0.elapsed_time(e) for e in ends) / reps)
                    continue
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
    # every build must produce the same images (byte for byte) as the in-tree one
    for c in cfgs:
        cfg = scenes.CONFIGS[c]
        sa = cfg.scene().to_abi()
        ref = None
        for name, L in libs.items():
            abi.check(L.rt_set_scene(ctxs[name], ctypes.byref(sa)), "rt_set_scene")
            o32 = torch.empty((cfg.height, cfg.width, 4), dtype=torch.float32, device="cuda")
            o8 = torch.empty((cfg.height, cfg.width, 4), dtype=torch.uint8, device="cuda")
            abi.check(L.rt_render_dev(ctxs[name], ctypes.byref(cfg.camera()), cfg.width, cfg.height, cfg.depth, None,
                                      ctypes.c_void_p(o32.data_ptr()), ctypes.c_void_p(o8.data_ptr()), None, None,
                                      ctypes.c_void_p(st.cuda_stream)), "rt_render_dev")
            torch.cuda.synchronize()
            if ref is None:
                ref = (o32, o8)
            elif not (torch.equal(o32, ref[0]) and torch.equal(o8, ref[1])):
                print(json.dumps({"config": c, "lib": name, "error": "image differs from base"}), flush=True)
    for (c, name), v in res.items():
        base = statistics.median(res[(c, "base")])
        med = statistics.median(v)
        print(json.dumps({"config": c, "lib": name, "median_ms": round(med, 4), "min_ms": round(min(v), 4),
                          "vs_base": round(med / base - 1, 4)}))
    for name, L in libs.items():
        L.rt_ctx_destroy(ctxs[name])
        for c in fly_ctx[name]:
            L.rt_ctx_destroy(c)


if __name__ == "__main__":
    main()
