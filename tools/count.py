#!/usr/bin/env python3
"""One c2-sized frame of a scene variant, for exact PMC instruction counts per variant
(rocprofv3 --pmc SQ_INSTS_VALU ... -- python3 tools/count.py VARIANT).  Variants: full, d0, nospheres,
noboard, empty, nolights."""
import dataclasses
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from ray_tracer_fragment_shader_amd import scenes  # noqa: E402
from ray_tracer_fragment_shader_amd.tracer import Tracer  # noqa: E402


def main():
    v = sys.argv[1] if len(sys.argv) > 1 else "full"
    cfg = scenes.CONFIGS[sys.argv[2] if len(sys.argv) > 2 else "c2"]
    sc, depth = cfg.scene(), cfg.depth
    if v == "d0":
        depth = 0
    elif v == "nospheres":
        sc = dataclasses.replace(sc, spheres=[])
    elif v == "noboard":
        sc = dataclasses.replace(sc, has_board=False)
    elif v == "empty":
        sc = dataclasses.replace(sc, spheres=[], has_board=False)
    elif v == "nolights":
        sc = dataclasses.replace(sc, lights=[])
    t = Tracer(0)
    t.set_scene(sc)
    bufs = t.alloc(cfg.width, cfg.height, rgba32f=True, rgba8=True)
    # first render, calibration, then cached renders of the view: the PMC mean per dispatch is the cached frames'
    for _ in range(int(os.environ.get("COUNT_FRAMES", "23"))):
        t.render_into(cfg.camera(), cfg.width, cfg.height, depth, bufs)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
