#!/usr/bin/env python3
"""What would compacting live rays across a 256-thread workgroup buy? (an LDS ray queue that
refills the bounce levels' waves.)  Renders a config once with per-pixel ray counters (rt_render_dev raycount: the
levels each pixel traced follow from its shadow-ray count), then counts, per bounce level, the wave-instructions'
worth of work the one-wave 8 x 8 tiles issue — waves with any live lane run the level's closest-hit code, waves with
any hit lane its shading — against the same work with each 32 x 8 workgroup's live rays packed into
ceil(live / 64) full waves.  Prints one JSON line per config.
usage: compaction_sim.py [c2,c3,c5]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from ray_tracer_fragment_shader_amd import scenes  # noqa: E402
from ray_tracer_fragment_shader_amd.tracer import Tracer  # noqa: E402


def levels_of(name):
    cfg = scenes.CONFIGS[name]
    t = Tracer(0)
    t.set_scene(cfg.scene())
    b = t.render(cfg.camera(), cfg.width, cfg.height, cfg.depth, rgba32f=False, raycount=True)
    torch.cuda.synchronize()
    rc = b["raycount"].cpu().numpy().view(np.uint32)
    t.close()
    return (rc >> 16) // cfg.n_lights, cfg.depth          # hits per pixel = levels traced past a hit


def simulate(lev, B):
    H, W = lev.shape
    Hp, Wp = (H + 7) // 8 * 8, (W + 31) // 32 * 32
    L = np.full((Hp, Wp), -1, np.int32)
    L[:H, :W] = lev
    tiles = L.reshape(Hp // 8, 8, Wp // 8, 8).transpose(0, 2, 1, 3).reshape(-1, 64)
    wg = L.reshape(Hp // 8, 8, Wp // 32, 32).transpose(0, 2, 1, 3).reshape(-1, 256)
    out = []
    for lvl in range(B + 1):
        alive_t = tiles >= (lvl if lvl else 0)
        hit_t = tiles >= lvl + 1
        alive_w = (wg >= (lvl if lvl else 0)).sum(1)
        hit_w = (wg >= lvl + 1).sum(1)
        out.append({"level": lvl,
                    "closest_hit_waves": int(alive_t.any(1).sum()), "closest_hit_waves_packed": int(np.ceil(alive_w / 64).sum()),
                    "closest_hit_lane_util": round(float(alive_t.sum() / 64 / max(alive_t.any(1).sum(), 1)), 3),
                    "shade_waves": int(hit_t.any(1).sum()), "shade_waves_packed": int(np.ceil(hit_w / 64).sum()),
                    "shade_lane_util": round(float(hit_t.sum() / 64 / max(hit_t.any(1).sum(), 1)), 3)})
    return out


def main():
    for name in (sys.argv[1].split(",") if len(sys.argv) > 1 else ["c2", "c3", "c5"]):
        lev, B = levels_of(name)
        per = simulate(lev, B)
        ch = sum(p["closest_hit_waves"] for p in per[1:])
        chp = sum(p["closest_hit_waves_packed"] for p in per[1:])
        sh = sum(p["shade_waves"] for p in per)
        shp = sum(p["shade_waves_packed"] for p in per)
        print(json.dumps({"config": name, "levels_hist": np.bincount(lev.ravel()).tolist(), "per_level": per,
                          "secondary_closest_hit_waves": [ch, chp], "shade_waves": [sh, shp],
                          "saved_fraction_secondary_closest_hit": round(1 - chp / max(ch, 1), 4),
                          "saved_fraction_shade": round(1 - shp / max(sh, 1), 4)}))


if __name__ == "__main__":
    main()
