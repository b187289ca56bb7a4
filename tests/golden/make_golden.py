#!/usr/bin/env python3
"""Generate the golden fixtures in tests/golden/ from the REFERENCE's own code.

Every expected value below is produced by oracle/_ref/libref.so: the hot-path source ranges of
/root/reference/Hw4/MySdlApplication.cpp compiled where they lie (oracle/Makefile, target `ref`) plus
oracle/ref_harness.cpp, which builds scenes with the reference classes and calls the reference
rayTraceRay / Shape::intersection.  Only inputs (rays, pixel coordinates) come from this script.

Outputs (all small, committed):
  frames_<cfg>.npz   160x120 full frame (float64 RGB, pitch 500/160) + 4096 sampled pixels of the
                     full-resolution frame (i, j, float64 RGB)
  kat_<scene>.npz    primitive known-answer tests: rays -> Shape::intersection (hit, material, point,
                     normal, reflected and transmitted ends) and rayTraceRay colours at depth 0..5
  manifest.json      FNV-1a 64 of every full-resolution float64 frame, image sizes, provenance
  tree_<scene>.npz   ray-tree scenes (scenes.TREE_CASES: partially transparent materials set into the
                     reference's material globals): small frame, sampled pixels, KAT colours; `--tree`
                     regenerates only these

Run in the build container (needs /root/reference):  python tests/golden/make_golden.py
"""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import pyoracle as po  # noqa: E402
from ray_tracer_fragment_shader_amd import scenes  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))
SMALL_W, SMALL_H = 160, 120
N_SAMPLES = 4096
CFGS = ["c1", "c2", "c3", "c5", "demo"]


def sample_pixels(cfg, rng):
    W, H = cfg.width, cfg.height
    pi = rng.integers(0, W, N_SAMPLES).astype(np.int32)
    pj = rng.integers(0, H, N_SAMPLES).astype(np.int32)
    # always include the corners and the centre
    pi[:5] = [0, W - 1, 0, W - 1, W // 2]
    pj[:5] = [0, 0, H - 1, H - 1, H // 2]
    return pi, pj


def kat_rays(scene, rng):
    """Rays exercising every branch of the intersection code (world coordinates)."""
    cam = np.array([0.0, 100.0, 200.0])
    starts, ends, tags = [], [], []

    def add(s, e, tag):
        starts.append(np.asarray(s, np.float64))
        ends.append(np.asarray(e, np.float64))
        tags.append(tag)

    centres = [np.array(sp.center()) + np.array([0.0, 0.0, -160.0]) for sp in scene.spheres]
    radii = [sp.radius for sp in scene.spheres]
    # meshes: centre, vertices, edge midpoints, face interiors, from inside, grazing the bounding sphere
    from ray_tracer_fragment_shader_amd.scenes import convert_string_coordinate
    for m in scene.meshes:
        c = np.array(convert_string_coordinate(m.square)) + np.array([0.0, 0.0, -160.0])
        h = m.edge / 2
        add(cam, c, "mesh_centre")
        add(c, c + np.array([0.3, 1.0, -0.2]), "inside_mesh")
        add(c, c + np.array([-1.0, -0.1, 0.05]), "inside_mesh")
        for sx in (-1, 1):
            for sy in (-1, 1):
                for sz in (-1, 1):
                    add(cam, c + h * np.array([sx, sy, sz]), "mesh_vertex")
                    add(cam, c + 0.999 * h * np.array([sx, sy, sz]), "mesh_near_vertex")
        for k in range(24):
            add(cam, c + rng.uniform(-h, h, 3), "mesh_interior")
        rb = np.sqrt(3.0) * m.edge / 2
        add(cam, c + np.array([rb, 0, 0]) * (1 - 1e-9), "mesh_bound_graze")
        add(c + np.array([0.0, 3 * h, 0.0]), c + np.array([0.0, -3 * h, 0.0]), "mesh_vertical")
    for c, r in zip(centres, radii):
        add(cam, c, "sphere_centre")
        add(c, c + np.array([1.0, 0.3, 0.2]), "inside_sphere")
        top = c + np.array([0.0, r, 0.0])
        add(top, top + np.array([0.0, 1.0, 0.0]), "on_surface_outward")
        add(top, top + np.array([0.0, -1.0, 0.0]), "on_surface_inward")
        d = c - cam
        d /= np.linalg.norm(d)
        perp = np.cross(d, np.array([0.0, 1.0, 0.0]))
        perp /= np.linalg.norm(perp)
        for f in (1.0 - 1e-9, 1.0, 1.0 + 1e-9, 0.999, 1.001):
            add(cam, c + f * r * perp, "grazing")
        add(cam, cam - d, "away")
    # board: corners, edges, square boundaries, the T1/T2 diagonal, checker parity
    for x in (-160.0, -159.9999, -120.0, -40.0, 0.0, 0.00001, 40.0, 80.0, 120.0, 159.9999, 160.0, 160.0001):
        for z in (0.0, -0.0001, -40.0, -160.0, -200.0, -280.0, -320.0, -319.9999, -320.0001):
            add(cam, np.array([x, 0.0, z]), "board_grid")
    for t in np.linspace(0.0, 1.0, 17):
        p = np.array([-160.0 + 320.0 * t, 0.0, -320.0 + 320.0 * t])      # diagonal P1 -> P3
        add(cam, p, "board_diagonal")
        add(cam, p + np.array([1e-7, 0.0, -1e-7]), "board_diagonal_eps")
    # parallel to the board plane, just above / on it
    add(np.array([-200.0, 1e-5, -100.0]), np.array([200.0, 1e-5, -100.0]), "parallel")
    add(np.array([-200.0, 0.0, -100.0]), np.array([200.0, 0.0, -100.0]), "in_plane")
    # bounding-sphere cull: far rays missing it, rays starting inside, on its surface
    add(np.array([0.0, 1000.0, 0.0]), np.array([1000.0, 1000.0, 0.0]), "bound_miss")
    add(np.array([0.0, 0.0, -160.0]), np.array([0.0, 10.0, -150.0]), "bound_inside")
    rb = np.sqrt(3.0) * 160.0
    add(np.array([0.0, rb, -160.0]), np.array([0.0, rb + 1.0, -160.0]), "bound_surface")
    # shadow-ray geometry: from board points to both light positions
    lights = [np.array(lt.position()) for lt in scene.lights] or [np.array([60.0, 200.0, -60.0])]
    for _ in range(96):
        p = np.array([rng.uniform(-160, 160), 0.0, rng.uniform(-320, 0)])
        for L in lights:
            add(p, L, "shadow")
    # random primary-like rays and random rays from random origins
    for _ in range(256):
        add(cam, np.array([rng.uniform(-250, 250), rng.uniform(-50, 150), rng.uniform(-400, 50)]), "random_cam")
    for _ in range(256):
        s = rng.uniform(-300, 300, 3)
        add(s, s + rng.normal(size=3) * rng.uniform(0.1, 50), "random")
    return np.array(starts), np.array(ends), np.array(tags)


def main() -> None:
    po.build(ref=True)
    rng = np.random.default_rng(20260415)
    manifest = {"generator": "tests/golden/make_golden.py",
                "reference": "oracle/_ref/libref.so = /root/reference/Hw4/MySdlApplication.cpp ranges "
                             "31-52,136-591,607-1249,1326-1346 + oracle/ref_harness.cpp",
                "hash": "FNV-1a 64 over the float64 RGB frame, pixel (i,j) at (j*W+i)*3, j=0 bottom row",
                "frames": {}}
    for name in CFGS:
        cfg = scenes.CONFIGS[name]
        sc = cfg.scene()
        t0 = time.time()
        small = po.ref_render(sc, SMALL_W, SMALL_H, cfg.depth, 500.0 / SMALL_W)
        pi, pj = sample_pixels(cfg, rng)
        samp = po.ref_render_pixels(sc, cfg.width, cfg.height, cfg.depth, cfg.pitch, pi, pj)
        full = po.ref_render(sc, cfg.width, cfg.height, cfg.depth, cfg.pitch)
        h = po.fnv1a64(full)
        np.savez_compressed(os.path.join(OUT, f"frames_{name}.npz"), small=small, pi=pi, pj=pj, samples=samp,
                            small_wh=np.array([SMALL_W, SMALL_H]), depth=np.array(cfg.depth))
        manifest["frames"][name] = {"width": cfg.width, "height": cfg.height, "depth": cfg.depth,
                                    "n_spheres": cfg.n_spheres, "n_lights": cfg.n_lights,
                                    "fnv1a64": f"{h:016x}", "max": float(full.max()),
                                    "nonzero_pixels": int((full.sum(axis=2) > 0).sum())}
        del full
        print(f"{name}: frames in {time.time() - t0:.1f}s hash {h:016x}", flush=True)
    for name in ("c3", "c5", "demo"):
        cfg = scenes.CONFIGS[name]
        sc = cfg.scene()
        starts, ends, tags = kat_rays(sc, rng)
        inter = po.ref_intersect(sc, starts, ends)
        colors = np.stack([po.ref_trace_rays(sc, starts, ends, d) for d in range(6)])
        np.savez_compressed(os.path.join(OUT, f"kat_{name}.npz"), starts=starts, ends=ends, tags=tags,
                            hit=inter["hit"], material=inter["material"], point=inter["point"],
                            normal=inter["normal"], reflected_end=inter["reflected_end"],
                            transmitted_end=inter["transmitted_end"], colors=colors)
        print(f"kat_{name}: {len(starts)} rays, {int(inter['hit'].sum())} hits", flush=True)
    make_tree(manifest)
    with open(os.path.join(OUT, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)


def canonical_nan(a: np.ndarray) -> np.ndarray:
    """NaN payloads are not part of the parity contract (the reference's own NaNs come from Line(p, p) on
    total internal reflection): every NaN becomes the default quiet NaN before hashing."""
    a = np.array(a, np.float64, copy=True)
    a[np.isnan(a)] = np.nan
    return a


def make_tree(manifest) -> None:
    """Ray-tree fixtures (scenes.TREE_CASES): materials that transmit AND reflect, set into the reference's
    own material globals (oracle/ref_harness.cpp ref_set_materials).  tree_<name>.npz: 160x120 frame,
    4096 sampled pixels of the full-size frame, KAT rays' rayTraceRay colours at depth 0..depth; the
    manifest holds the FNV-1a of the full-size frame with NaNs made canonical."""
    rng = np.random.default_rng(20261016)
    manifest.setdefault("tree", {})
    for name in scenes.TREE_CASES:
        sc, cfg, depth, (W, H) = scenes.tree_case(name)
        t0 = time.time()
        small = po.ref_render(sc, SMALL_W, SMALL_H, depth, 500.0 / SMALL_W)
        pi = rng.integers(0, W, N_SAMPLES).astype(np.int32)
        pj = rng.integers(0, H, N_SAMPLES).astype(np.int32)
        samp = po.ref_render_pixels(sc, W, H, depth, 500.0 / W, pi, pj)
        full = po.ref_render(sc, W, H, depth, 500.0 / W)
        h = po.fnv1a64(canonical_nan(full))
        starts, ends, tags = kat_rays(sc, rng)
        colors = np.stack([po.ref_trace_rays(sc, starts, ends, d) for d in range(depth + 1)])
        np.savez_compressed(os.path.join(OUT, f"tree_{name[5:]}.npz"), small=small, pi=pi, pj=pj, samples=samp,
                            small_wh=np.array([SMALL_W, SMALL_H]), depth=np.array(depth), starts=starts, ends=ends,
                            tags=tags, colors=colors, wh=np.array([W, H]))
        manifest["tree"][name] = {"width": W, "height": H, "depth": depth, "fnv1a64_canonical_nan": f"{h:016x}",
                                  "nan_pixels": int(np.isnan(full).any(axis=2).sum()),
                                  "materials": {str(k): [list(v) if isinstance(v, tuple) else v for v in m]
                                                for k, m in scenes.TREE_CASES[name][1].items()}}
        del full
        print(f"{name}: {time.time() - t0:.1f}s hash {h:016x}", flush=True)


if __name__ == "__main__":
    if sys.argv[1:] == ["--tree"]:                  # only the ray-tree fixtures (the others unchanged)
        po.build(ref=True)
        path = os.path.join(OUT, "manifest.json")
        with open(path) as f:
            man = json.load(f)
        make_tree(man)
        with open(path, "w") as f:
            json.dump(man, f, indent=1, sort_keys=True)
    else:
        main()
