#!/usr/bin/env python3
"""Where a one-rank rt_render_multi frame (the c4 leg at N = 1) differs from a plain c3 render (0.146 vs
0.128 ms).  One process, three contexts on one stream, interleaved rounds; per mode the serial frame time from HIP
events around `n` back-to-back calls (device time) and from the wall clock with a synchronisation (host + device):
  dev8     rt_render_dev, RGBA8 only (the c4 leg's output)
  dev32_8  rt_render_dev, RGBA32F + RGBA8 (the bench's c3 config line)
  multi1   rt_render_multi of a one-rank RCCL group, RGBA8 (the c4 leg at N = 1)
Prints one JSON line: median ms per frame per mode and the host issue time per call."""
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
    L = abi.lib()
    cfg = scenes.CONFIGS["c3"]
    W, H, B = cfg.width, cfg.height, cfg.depth
    cam = cfg.camera()
    st = torch.cuda.current_stream()
    sp = ctypes.c_void_p(st.cuda_stream)
    tr = {m: Tracer(0) for m in ("dev8", "dev32_8", "multi1")}
    for t in tr.values():
        t.set_scene(cfg.scene())
    img8 = {m: torch.empty((H, W, 4), dtype=torch.uint8, device="cuda") for m in tr}
    img32 = torch.empty((H, W, 4), dtype=torch.float32, device="cuda")
    g = ctypes.c_void_p()
    arr = (ctypes.c_void_p * 1)(tr["multi1"]._ctx.value)
    abi.check(L.rt_group_create(arr, 1, abi.RT_TRANSPORT_RCCL, ctypes.byref(g)), "rt_group_create")
    calls = {
        "dev8": lambda: L.rt_render_dev(tr["dev8"]._ctx, ctypes.byref(cam), W, H, B, None, None,
                                        ctypes.c_void_p(img8["dev8"].data_ptr()), None, None, sp),
        "dev32_8": lambda: L.rt_render_dev(tr["dev32_8"]._ctx, ctypes.byref(cam), W, H, B, None,
                                           ctypes.c_void_p(img32.data_ptr()), ctypes.c_void_p(img8["dev32_8"].data_ptr()),
                                           None, None, sp),
        "multi1": lambda: L.rt_render_multi(g, ctypes.byref(cam), W, H, B, 0, abi.RT_OUT_RGBA8, None,
                                            ctypes.c_void_p(img8["multi1"].data_ptr()), sp),
    }
    for f in calls.values():
        for _ in range(5):
            abi.check(f(), "render")
    torch.cuda.synchronize()
    n = int(os.environ.get("N", "40"))
    dev = {m: [] for m in calls}
    wall = {m: [] for m in calls}
    issue = {m: [] for m in calls}
    for _ in range(int(os.environ.get("ROUNDS", "7"))):
        for m, f in calls.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            e0.record(st)
            for _ in range(n):
                f()
            e1.record(st)
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            dev[m].append(e0.elapsed_time(e1) / n)
            wall[m].append((t2 - t0) * 1e3 / n)
            issue[m].append((t1 - t0) * 1e6 / n)
    same = bool(torch.equal(img8["dev8"], img8["multi1"]) and torch.equal(img8["dev8"], img8["dev32_8"]))
    print(json.dumps({"config": "c3", "frames_per_round": n, "images_equal": same,
                      "dev_ms": {m: round(statistics.median(v), 5) for m, v in dev.items()},
                      "wall_ms": {m: round(statistics.median(v), 5) for m, v in wall.items()},
                      "issue_us_per_call": {m: round(statistics.median(v), 1) for m, v in issue.items()}}))
    L.rt_group_destroy(g)
    for t in tr.values():
        t.close()


if __name__ == "__main__":
    main()
