#!/usr/bin/env python3
"""Generate tests/golden/screen.json: pins of the reference-faithful rayTraceScreen
from the REFERENCE's own rayTraceScreen (oracle/_ref/libref.so: MySdlApplication.cpp:1251-1324 compiled
where it lies, its glBegin/glColor3d/glVertex2i/glEnd calls linked to the image's real libGL with no
context, where they do nothing).  The colours it hands to GL are therefore not observable; its rand()
consumption is (oracle/ref_harness.cpp ref_screen_rand_calls): 3 calls per jittered sample, i.e. the
sample counts that the convergence test and the colour carry-over produced.  Pinned per case:
  calls        rand() calls of the whole frame (glibc rand, srand(seed))
  row0_calls   calls of the first k pixels of the bottom row, k = 1..K (frames W = k, H = 1 with the full
               frame's bottom_x / bottom_y), i.e. the per-pixel sample counts of that row
Run in the build container (needs /root/reference):  python tests/golden/make_golden_screen.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import pyoracle as po  # noqa: E402
from ray_tracer_fragment_shader_amd import scenes  # noqa: E402

CASES = [("c1", 48, 36, 1), ("c2", 64, 36, 1), ("demo", 50, 50, 1), ("c2", 40, 30, 7)]
K = 40


def main():
    po.build(ref=True)
    out = {"generator": "tests/golden/make_golden_screen.py",
           "reference": "oracle/_ref/libref.so rayTraceScreen (MSA:1251-1324) + randomUnit (MSA:1148-1169), "
                        "glibc rand(); GL calls are no-ops (no context)",
           "depth": 5, "cases": []}
    for name, W, H, seed in CASES:
        sc = scenes.CONFIGS[name].scene()
        bx, by = -(W // 2), -(H // 2)
        calls = po.ref_screen_rand_calls(sc, W, H, bx, by, seed)
        row0 = [po.ref_screen_rand_calls(sc, k, 1, bx, by, seed) for k in range(1, K + 1)]
        out["cases"].append({"scene": name, "width": W, "height": H, "bottom_x": bx, "bottom_y": by,
                             "seed": seed, "calls": calls, "row0_calls": row0})
        print(name, W, H, seed, calls, flush=True)
    with open(os.path.join(ROOT, "tests", "golden", "screen.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
