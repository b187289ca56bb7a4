#!/usr/bin/env python3
"""Wave-level event counts of one frame per config (needs an RT_COUNTERS=1 build of librt_amd.so, e.g.
`bash tools/variants.sh cnt=-DRT_COUNTERS=1` and LIB=tools/_var/cnt/librt_amd.so): per-wave culling masks and how
many spheres they keep, exact sphere tests run by a wave, bounce levels.  Prints one JSON line per config."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from ray_tracer_fragment_shader_amd import abi, scenes  # noqa: E402

NAMES = ["waves", "cone_kept", "ray_masks", "ray_kept", "shadow_masks", "shadow_kept", "exact_ray", "exact_shadow",
         "board_shadow", "levels", "exact_primary", "filter_ray", "filter_shadow",
         "lanes_filter_ray", "lanes_exact_ray", "lanes_filter_shadow", "lanes_exact_shadow", "lanes_level_alive",
         "lanes_level_hit"]
# lane utilisation of an event = its lanes / (64 x its count)
UTIL = {"filter_ray": "lanes_filter_ray", "exact_ray": "lanes_exact_ray", "filter_shadow": "lanes_filter_shadow",
        "exact_shadow": "lanes_exact_shadow", "levels": "lanes_level_alive"}
path = os.environ.get("LIB", os.path.join(ROOT, "tools", "_var", "cnt", "librt_amd.so"))
L = ctypes.CDLL(path)
for fn, (res, args) in abi.SIGNATURES.items():
    if hasattr(L, fn):
        getattr(L, fn).restype = res
        getattr(L, fn).argtypes = args
L.rt_debug_counters.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
for name in (sys.argv[1].split(",") if len(sys.argv) > 1 else ["c2", "c3", "c5"]):
    cfg = scenes.CONFIGS[name]
    ctx = ctypes.c_void_p()
    abi.check(L.rt_ctx_create(0, ctypes.byref(ctx)), "ctx")
    sa = cfg.scene().to_abi()
    abi.check(L.rt_set_scene(ctx, ctypes.byref(sa)), "scene")
    cnt = torch.zeros(len(NAMES), dtype=torch.int64, device="cuda")
    abi.check(L.rt_debug_counters(ctx, ctypes.c_void_p(cnt.data_ptr())), "counters")
    cam = cfg.camera()
    o8 = torch.empty((cfg.height, cfg.width, 4), dtype=torch.uint8, device="cuda")
    abi.check(L.rt_render_dev(ctx, ctypes.byref(cam), cfg.width, cfg.height, cfg.depth, None, None,
                              ctypes.c_void_p(o8.data_ptr()), None, None, None), "render")
    torch.cuda.synchronize()
    v = dict(zip(NAMES, cnt.cpu().tolist()))
    w = max(v["waves"], 1)
    util = {f"util_{k}": round(v[u] / 64 / max(v[k], 1), 3) for k, u in UTIL.items()}
    util["util_level_hit"] = round(v["lanes_level_hit"] / 64 / max(v["levels"], 1), 3)
    print(json.dumps({"config": name, **v, **{f"{k}_per_wave": round(v[k] / w, 3) for k in NAMES[1:]}, **util}),
          flush=True)
    L.rt_ctx_destroy(ctx)
