#!/usr/bin/env python3
"""profiles/pmc_<config>.json (read by bench.py's roofline.traffic) from a tools/pmc.sh summary.json.
usage: pmc_profile.py <summary.json> <config> [note]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from ray_tracer_fragment_shader_amd import scenes  # noqa: E402


def main(path, config, note=""):
    d = json.load(open(path))
    k = next(n for n in d if n.startswith("rt_render_kernel"))
    c = d[k]
    cfg = scenes.CONFIGS[config]
    out = {
        "config": config,
        "kernel": k,
        "source": "rocprofv3 --pmc WRITE_SIZE / FETCH_SIZE, separate passes (tools/pmc.sh), mean per dispatch",
        "write_size_kib": c["WRITE_SIZE"],
        "fetch_size_kib": c["FETCH_SIZE"],
        "correction": "gfx950 FETCH_SIZE counts half of wide coalesced reads (MI355X_MICROARCH.md HBM): read "
                      "bytes = 2 x FETCH_SIZE; WRITE_SIZE exact for 16-B/lane stores",
        "hbm_bytes_per_launch": c["WRITE_SIZE"] * 1024 + 2 * c["FETCH_SIZE"] * 1024,
        "algorithmic_bytes_per_launch": cfg.width * cfg.height * 20,
    }
    if note:
        out["note"] = note
    with open(os.path.join(ROOT, "profiles", f"pmc_{config}.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main(*sys.argv[1:])
