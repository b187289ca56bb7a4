#!/usr/bin/env python3
"""draw()'s pipelined host frames at c2 (GRAY8, pinned), for a rocprofv3 --kernel-trace timeline: K frames of
rt_render_packed_async, waiting for frame f - DEPTH after queueing frame f (RT_COPY_MODE / RT_COPY_BLOCKS from the
environment).  With `parse <dir>`: per-frame render and copy kernel spans, how much of each copy overlaps a
render, and the gaps on each queue."""
import csv
import ctypes
import glob
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run():
    import torch  # noqa: F401
    from ray_tracer_fragment_shader_amd import abi, scenes
    from ray_tracer_fragment_shader_amd.tracer import Tracer
    L = abi.lib()
    cfg = scenes.CONFIGS["c2"]
    W, H, B = cfg.width, cfg.height, cfg.depth
    sa, cam = cfg.scene().to_abi(), cfg.camera()
    t = Tracer(0)
    pins = []
    for _ in range(3):
        p = ctypes.c_void_p()
        abi.check(L.rt_host_alloc(W * H, ctypes.byref(p)), "rt_host_alloc")
        pins.append(p)
    a = (t._ctx, ctypes.byref(sa), ctypes.byref(cam), W, H, B, abi.RT_PIXEL_GRAY8)
    depth = int(os.environ.get("DEPTH", "1"))
    k = int(os.environ.get("K", "40"))
    tk = [ctypes.c_uint64() for _ in range(3)]
    for f in range(10):
        abi.check(L.rt_render_packed_async(*a, pins[f % 3], ctypes.byref(tk[f % 3])), "async")
    abi.check(L.rt_ctx_wait(t._ctx, 0), "wait")
    t0 = time.perf_counter()
    for f in range(k):
        abi.check(L.rt_render_packed_async(*a, pins[f % 3], ctypes.byref(tk[f % 3])), "async")
        if f >= depth:
            abi.check(L.rt_ctx_wait(t._ctx, tk[(f - depth) % 3].value), "wait")
    abi.check(L.rt_ctx_wait(t._ctx, 0), "wait")
    print(json.dumps({"us_per_frame": round((time.perf_counter() - t0) / k * 1e6, 1), "depth": depth,
                      "mode": os.environ.get("RT_COPY_MODE"), "blocks": os.environ.get("RT_COPY_BLOCKS")}))
    for p in pins:
        L.rt_host_free(p)


def parse(d):
    f = glob.glob(d + "/**/*kernel_trace.csv", recursive=True)[0]
    rows = list(csv.DictReader(open(f)))
    ren = sorted([(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows
                  if "rt_render_kernel" in r["Kernel_Name"]])[-30:]
    cop = sorted([(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows
                  if "rt_copy_out_kernel" in r["Kernel_Name"] or "copyBuffer" in r["Kernel_Name"]])[-30:]
    mc = glob.glob(d + "/**/*memory_copy_trace.csv", recursive=True)
    if not cop and mc:                                       # SDMA copies (--memory-copy-trace)
        cop = sorted([(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in csv.DictReader(open(mc[0]))
                      if "DEVICE_TO_HOST" in r.get("Direction", "")])[-30:]
    lo = max(ren[0][0], cop[0][0])
    ren = [x for x in ren if x[0] >= lo]
    cop = [x for x in cop if x[0] >= lo]

    def overlap(c):
        return sum(max(0, min(c[1], r[1]) - max(c[0], r[0])) for r in ren)
    out = {"render_us": round(statistics.median((e - s) / 1e3 for s, e in ren), 2),
           "copy_us": round(statistics.median((e - s) / 1e3 for s, e in cop), 2),
           "copy_overlapped_frac": round(statistics.median(overlap(c) / max(1, c[1] - c[0]) for c in cop), 3),
           "render_gap_us": round(statistics.median((ren[i + 1][0] - ren[i][1]) / 1e3 for i in range(len(ren) - 1)), 2),
           "copy_start_after_render_end_us": round(statistics.median(
               min((c[0] - r[1]) / 1e3 for r in ren if r[1] <= c[0] + 1) for c in cop if any(r[1] <= c[0] + 1 for r in ren)), 2),
           "period_us": round((ren[-1][0] - ren[0][0]) / 1e3 / (len(ren) - 1), 2)}
    print(json.dumps(out))


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "parse":
        parse(sys.argv[2])
    else:
        run()
