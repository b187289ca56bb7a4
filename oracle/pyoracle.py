"""Python loader for the oracle libraries.  TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module; the
product package never does.

* ``librt_oracle.so`` — the C restatement (oracle/rt_oracle.c), runs anywhere (also on the GPU box).
* ``_ref/libref.so``  — the reference's own rayTraceRay compiled from /root/reference (oracle/Makefile
  target ``ref``); exists only in the build container, never on the GPU box.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from ctypes import POINTER, c_char_p, c_double, c_int, c_int32, c_uint32, c_uint64, c_void_p, c_size_t

import numpy as np

from ray_tracer_fragment_shader_amd import abi

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "librt_oracle.so")
REF_SO = os.path.join(HERE, "_ref", "libref.so")
REF_SRC = "/root/reference/Hw4/MySdlApplication.cpp"

_oracle = None
_ref = None


def build(ref: bool = True) -> None:
    """make the restatement (always) and the reference build (when /root/reference is present)."""
    subprocess.run(["make", "-C", HERE, "all"], check=True, stdout=subprocess.DEVNULL)
    if ref and os.path.exists(REF_SRC):
        subprocess.run(["make", "-C", HERE, "ref"], check=True, stdout=subprocess.DEVNULL)


def oracle() -> ctypes.CDLL:
    global _oracle
    if _oracle is None:
        if not os.path.exists(ORACLE_SO):
            build(ref=False)
        L = ctypes.CDLL(ORACLE_SO)
        L.oracle_render.restype = c_int
        L.oracle_render.argtypes = [POINTER(abi.rt_scene), POINTER(abi.rt_camera), c_int, c_int, c_int,
                                    POINTER(abi.rt_rows), c_void_p, c_void_p, c_int]
        L.oracle_trace_rays.restype = c_int
        L.oracle_trace_rays.argtypes = [POINTER(abi.rt_scene), c_void_p, c_void_p, c_int, c_int, c_void_p,
                                        c_void_p, c_int]
        L.oracle_intersect.restype = c_int
        L.oracle_intersect.argtypes = [POINTER(abi.rt_scene), c_void_p, c_void_p, c_int, POINTER(abi.rt_hit)]
        L.oracle_camera_basis.restype = None
        L.oracle_camera_basis.argtypes = [POINTER(abi.rt_camera), c_void_p, c_void_p]
        L.oracle_local_rows.restype = c_int
        L.oracle_local_rows.argtypes = [c_int, POINTER(abi.rt_rows)]
        L.oracle_convert_string_coordinate.restype = None
        L.oracle_convert_string_coordinate.argtypes = [c_char_p, c_void_p]
        L.oracle_fnv1a64.restype = c_uint64
        L.oracle_fnv1a64.argtypes = [c_void_p, c_size_t]
        L.oracle_render_screen.restype = c_int
        L.oracle_render_screen.argtypes = [POINTER(abi.rt_scene), c_void_p, c_void_p, c_void_p, c_int, c_int, c_int,
                                           c_int, c_int, c_int, ctypes.c_uint32, c_void_p, c_void_p, c_void_p]
        L.oracle_rand_sequence.restype = None
        L.oracle_rand_sequence.argtypes = [c_int, ctypes.c_uint32, c_int, c_void_p]
        _oracle = L
    return _oracle


def ref_available() -> bool:
    return os.path.exists(REF_SO) or os.path.exists(REF_SRC)


def ref() -> ctypes.CDLL:
    global _ref
    if _ref is None:
        if not os.path.exists(REF_SO):
            if not os.path.exists(REF_SRC):
                raise RuntimeError("reference build unavailable (no /root/reference here)")
            build(ref=True)
        L = ctypes.CDLL(REF_SO)
        scene_args = [c_char_p, c_int, c_void_p, c_void_p, c_void_p, c_char_p, c_void_p, c_int]
        L.ref_render.restype = c_int
        L.ref_render.argtypes = scene_args + [c_int, c_int, c_int, c_double, c_int, c_int, c_void_p, c_int]
        L.ref_render_pixels.restype = c_int
        L.ref_render_pixels.argtypes = scene_args + [c_int, c_int, c_int, c_double, c_void_p, c_void_p, c_int,
                                                     c_void_p, c_int]
        L.ref_trace_rays.restype = c_int
        L.ref_trace_rays.argtypes = scene_args + [c_void_p, c_void_p, c_int, c_int, c_void_p]
        L.ref_intersect.restype = c_int
        L.ref_intersect.argtypes = [c_char_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int,
                                    c_void_p, c_void_p, c_void_p]
        L.ref_convert_string_coordinate.restype = None
        L.ref_convert_string_coordinate.argtypes = [c_char_p, c_void_p]
        L.ref_set_materials.restype = None
        L.ref_set_materials.argtypes = [c_void_p]
        L.ref_default_materials.restype = None
        L.ref_default_materials.argtypes = [c_void_p]
        L.ref_screen_rand_calls.restype = c_uint64
        L.ref_screen_rand_calls.argtypes = scene_args + [c_int, c_int, c_int, c_int, ctypes.c_uint, c_uint64]
        _ref = L
    return _ref


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


def fnv1a64(a: np.ndarray) -> int:
    a = np.ascontiguousarray(a)
    return int(oracle().oracle_fnv1a64(_ptr(a), a.nbytes))


# ---------------------------------------------------------------------------------------- restatement
def render(scene_abi, cam, width, height, depth, rows=None, nthreads=0):
    """-> (rgb float64 [local_rows, W, 3], raycount uint32 [local_rows, W])"""
    L = oracle()
    nl = L.oracle_local_rows(height, ctypes.byref(rows) if rows is not None else None)
    rgb = np.zeros((nl, width, 3), np.float64)
    rc = np.zeros((nl, width), np.uint32)
    code = L.oracle_render(ctypes.byref(scene_abi), ctypes.byref(cam), width, height, depth,
                           ctypes.byref(rows) if rows is not None else None, _ptr(rgb), _ptr(rc), nthreads)
    if code:
        raise RuntimeError(f"oracle_render failed: {code}")
    return rgb, rc


def trace_rays(scene_abi, starts, ends, depth, nthreads=0):
    starts = np.ascontiguousarray(starts, np.float64)
    ends = np.ascontiguousarray(ends, np.float64)
    n = starts.shape[0]
    rgb = np.zeros((n, 3), np.float64)
    rc = np.zeros(n, np.uint32)
    code = oracle().oracle_trace_rays(ctypes.byref(scene_abi), _ptr(starts), _ptr(ends), n, depth, _ptr(rgb),
                                      _ptr(rc), nthreads)
    if code:
        raise RuntimeError(f"oracle_trace_rays failed: {code}")
    return rgb, rc


def intersect(scene_abi, starts, ends):
    """-> dict of arrays: hit, material, point, normal, reflected_end"""
    starts = np.ascontiguousarray(starts, np.float64)
    ends = np.ascontiguousarray(ends, np.float64)
    n = starts.shape[0]
    hits = (abi.rt_hit * max(n, 1))()
    code = oracle().oracle_intersect(ctypes.byref(scene_abi), _ptr(starts), _ptr(ends), n, hits)
    if code:
        raise RuntimeError(f"oracle_intersect failed: {code}")
    return hits_to_dict(hits, n)


def hits_to_dict(hits, n):
    raw = np.frombuffer(hits, dtype=np.uint8, count=n * ctypes.sizeof(abi.rt_hit)).reshape(n, -1)
    d = raw[:, :96].copy().view(np.float64).reshape(n, 12)
    i = raw[:, 96:104].copy().view(np.int32).reshape(n, 2)
    return {"point": d[:, 0:3], "normal": d[:, 3:6], "reflected_end": d[:, 6:9], "transmitted_end": d[:, 9:12],
            "hit": i[:, 0], "material": i[:, 1]}


def camera_basis(cam):
    r = np.zeros(3)
    u = np.zeros(3)
    oracle().oracle_camera_basis(ctypes.byref(cam), _ptr(r), _ptr(u))
    return r, u


def screen_points(cam, width, height, rows=None):
    """Primary-ray end points sp(i, j) of SURVEY.md Appendix B, computed with numpy in the same operation
    order (IEEE float64, elementwise: bit-identical to the C code)."""
    right, upp = camera_basis(cam)
    look = np.array(cam.look_at[:])
    js = np.arange(height)
    if rows is not None and rows.n_ranks > 1:
        js = js[(js // rows.band_height) % rows.n_ranks == rows.rank]
    ii = np.arange(width)
    a = cam.pitch * (ii + cam.bottom_x).astype(np.float64)
    b = cam.pitch * (js + cam.bottom_y).astype(np.float64)
    sp = (look[None, None, :] + a[None, :, None] * right[None, None, :]) + b[:, None, None] * upp[None, None, :]
    return sp


# ------------------------------------------------------------------- reference-faithful rayTraceScreen
GLIBC, MSVC = 0, 1       # rand() generators (oracle_render_screen)
CAMERA = ((0.0, 100.0, 200.0), (0.0, 0.0, -160.0), (0.0, 1.0, 0.0))   # MSA:38-40


def render_screen(scene_abi, width, height, depth=5, rng=GLIBC, seed=1, bottom_x=None, bottom_y=None):
    """rayTraceScreen as the app runs it (jitter, <= 16 adaptive samples, colour carry-over; serial).
    Returns (rgb [H, W, 3] as handed to glColor3d, samples [H, W] uint8, rand() calls)."""
    bx = -(width // 2) if bottom_x is None else bottom_x
    by = -(height // 2) if bottom_y is None else bottom_y
    eye, look, up = (np.array(v, np.float64) for v in CAMERA)
    rgb = np.zeros((height, width, 3), np.float64)
    ns = np.zeros((height, width), np.uint8)
    calls = c_uint64()
    rc = oracle().oracle_render_screen(ctypes.byref(scene_abi), _ptr(eye), _ptr(look), _ptr(up), bx, by, width,
                                       height, depth, rng, seed, _ptr(rgb), _ptr(ns), ctypes.byref(calls))
    if rc:
        raise RuntimeError(f"oracle_render_screen failed: {rc}")
    return rgb, ns, int(calls.value)


def rand_sequence(rng, seed, n):
    out = np.zeros(n, np.int32)
    oracle().oracle_rand_sequence(rng, seed, n, _ptr(out))
    return out


def ref_screen_rand_calls(scene, width, height, bottom_x=None, bottom_y=None, seed=1, max_calls=1 << 32):
    """rand() calls made by the reference's own rayTraceScreen on this frame (glibc rand, MAX_DEPTH)."""
    bx = -(width // 2) if bottom_x is None else bottom_x
    by = -(height // 2) if bottom_y is None else bottom_y
    return int(_ref_scene(scene).ref_screen_rand_calls(*scene.ref_args(), width, height, bx, by, seed, max_calls))


# ------------------------------------------------------------------------------------- reference build
def _ref_scene(scene):
    """The reference library with its five material globals set to the scene's (every ref_* call: the
    scenes it builds copy them), -> the library."""
    L = ref()
    m = np.ascontiguousarray(scene.material_values(), np.float64)
    L.ref_set_materials(_ptr(m))
    return L


def ref_materials():
    """The reference's own material globals (5 x 13 doubles) as it initialised them (MSA:583-588)."""
    m = np.zeros(65, np.float64)
    ref().ref_default_materials(_ptr(m))
    return m


def ref_render(scene, width, height, depth, pitch, row_begin=0, row_end=None, nthreads=0):
    row_end = height if row_end is None else row_end
    rgb = np.zeros((row_end - row_begin, width, 3), np.float64)
    _ref_scene(scene).ref_render(*scene.ref_args(), width, height, depth, float(pitch), row_begin, row_end, _ptr(rgb),
                     nthreads)
    return rgb


def ref_render_pixels(scene, width, height, depth, pitch, pi, pj, nthreads=0):
    pi = np.ascontiguousarray(pi, np.int32)
    pj = np.ascontiguousarray(pj, np.int32)
    rgb = np.zeros((pi.shape[0], 3), np.float64)
    _ref_scene(scene).ref_render_pixels(*scene.ref_args(), width, height, depth, float(pitch), _ptr(pi), _ptr(pj),
                            pi.shape[0], _ptr(rgb), nthreads)
    return rgb


def ref_trace_rays(scene, starts, ends, depth):
    starts = np.ascontiguousarray(starts, np.float64)
    ends = np.ascontiguousarray(ends, np.float64)
    rgb = np.zeros((starts.shape[0], 3), np.float64)
    _ref_scene(scene).ref_trace_rays(*scene.ref_args(), _ptr(starts), _ptr(ends), starts.shape[0], depth, _ptr(rgb))
    return rgb


def ref_intersect(scene, starts, ends):
    starts = np.ascontiguousarray(starts, np.float64)
    ends = np.ascontiguousarray(ends, np.float64)
    n = starts.shape[0]
    out12 = np.zeros((n, 12), np.float64)
    hit = np.zeros(n, np.int32)
    mat = np.zeros(n, np.int32)
    a = scene.ref_args()
    _ref_scene(scene).ref_intersect(a[0], a[1], a[2], a[3], a[4], _ptr(starts), _ptr(ends), n, _ptr(out12), _ptr(hit),
                        _ptr(mat))
    return {"point": out12[:, 0:3], "normal": out12[:, 3:6], "reflected_end": out12[:, 6:9],
            "transmitted_end": out12[:, 9:12], "hit": hit, "material": mat}
