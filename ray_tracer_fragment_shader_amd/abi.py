"""ctypes mirror of include/rt_api.h and the loader for the in-tree librt_amd.so.

The shared library is the product (HIP kernels + C ABI).  There is no Python or CPU fallback: if the
library is missing, :func:`lib` raises; if no HIP device is present, every render call returns RT_EHIP
and :func:`check` raises :class:`RtError`.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, Structure, c_char_p, c_double, c_int, c_int32, c_uint8, c_uint32, c_uint64, c_void_p

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_DIR = os.path.join(_HERE, "lib")
# (RT_LIB_PATH: an experiment build of the same ABI, for the instruction-count tools; the product loads LIB_DIR's)
LIB_PATH = os.environ.get("RT_LIB_PATH") or os.path.join(LIB_DIR, "librt_amd.so")

RT_OK = 0
RT_EINVAL = -1
RT_EHIP = -2
RT_ENOMEM = -3
RT_EUNSUPPORTED = -4
RT_MAX_SPHERES = 1024
RT_MAX_LIGHTS = 16
RT_MAX_MESHES = 64
RT_MAX_DEPTH = 7
RT_RAND_GLIBC, RT_RAND_MSVC = 0, 1
RT_MESH_TETRAHEDRON = 1
RT_MESH_CUBE = 2
ABI_VERSION = 7
RT_TRANSPORT_AUTO, RT_TRANSPORT_RCCL, RT_TRANSPORT_COPY = -1, 0, 1
RT_OUT_RGBA32F, RT_OUT_RGBA8 = 1, 2
RT_PIXEL_RGBA32F, RT_PIXEL_GRAY32F, RT_PIXEL_RGBA8, RT_PIXEL_RGB8, RT_PIXEL_GRAY8 = 0, 1, 2, 3, 4
PIXEL_BYTES = {RT_PIXEL_RGBA32F: 16, RT_PIXEL_GRAY32F: 4, RT_PIXEL_RGBA8: 4, RT_PIXEL_RGB8: 3, RT_PIXEL_GRAY8: 1}
RT_COMM_ID_BYTES = 128

D3 = c_double * 3


class rt_material(Structure):
    _fields_ = [("ambient", D3), ("diffuse", D3), ("specular", D3), ("transparency", D3), ("refraction", c_double)]


class rt_sphere(Structure):
    _fields_ = [("center", D3), ("radius", c_double)]


class rt_light(Structure):
    _fields_ = [("color", D3), ("position", D3)]


class rt_mesh(Structure):
    _fields_ = [("kind", c_int32), ("after_spheres", c_int32), ("position", D3), ("edge", c_double)]


class rt_scene(Structure):
    _fields_ = [
        ("position", D3),
        ("radius", c_double),
        ("has_board", c_int32),
        ("n_spheres", c_int32),
        ("n_lights", c_int32),
        ("reserved0", c_int32),
        ("board_position", D3),
        ("board_half_size", c_double),
        ("square_edge_size", c_double),
        ("small_number", c_double),
        ("attenuation_factor", c_double),
        ("white_square", rt_material),
        ("black_square", rt_material),
        ("sphere_material", rt_material),
        ("spheres", POINTER(rt_sphere)),
        ("lights", POINTER(rt_light)),
        ("tetrahedron_material", rt_material),
        ("cube_material", rt_material),
        ("n_meshes", c_int32),
        ("reserved1", c_int32),
        ("meshes", POINTER(rt_mesh)),
    ]


class rt_camera(Structure):
    _fields_ = [("eye", D3), ("look_at", D3), ("up", D3), ("pitch", c_double), ("bottom_x", c_int32),
                ("bottom_y", c_int32)]


class rt_rows(Structure):
    _fields_ = [("band_height", c_int32), ("n_ranks", c_int32), ("rank", c_int32), ("frames", c_int32)]


class rt_stats(Structure):
    _fields_ = [("primary_rays", c_uint64), ("reflect_rays", c_uint64), ("shadow_rays", c_uint64),
                ("kernel_ms", c_double)]


class rt_hit(Structure):
    _fields_ = [("point", D3), ("normal", D3), ("reflected_end", D3), ("transmitted_end", D3), ("hit", c_int32),
                ("material", c_int32)]


class rt_group_stats(Structure):
    _fields_ = [("frames", c_int32), ("wire_float", c_int32), ("wire_byte", c_int32), ("ranks_timed", c_int32),
                ("payload_bytes", c_uint64), ("render_ms", c_double), ("gather_ms", c_double),
                ("assemble_ms", c_double), ("frame_ms", c_double)]


class rt_group_plan(Structure):
    _fields_ = [("n_ranks", c_int32), ("rank", c_int32), ("band_height", c_int32), ("slab_rows", c_int32),
                ("rank_rows", c_int32), ("wire", c_int32 * 2), ("elem_bytes", c_int32 * 2),
                ("slab_bytes", c_uint64 * 2), ("send_bytes", c_uint64 * 2), ("gather_bytes", c_uint64 * 2),
                ("payload_bytes", c_uint64), ("renderers", c_int32), ("root_renders", c_int32)]


class RtError(RuntimeError):
    def __init__(self, code: int, where: str, msg: str):
        super().__init__(f"{where}: rt error {code}: {msg}")
        self.code = code


# name -> (restype, argtypes); the exact set declared in include/rt_api.h
_P = POINTER
SIGNATURES = {
    "rt_abi_version": (c_int, []),
    "rt_last_error": (c_char_p, []),
    "rt_device_count": (c_int, [_P(c_int)]),
    "rt_ctx_create": (c_int, [c_int, _P(c_void_p)]),
    "rt_ctx_destroy": (c_int, [c_void_p]),
    "rt_scene_init_reference": (c_int, [_P(rt_scene)]),
    "rt_convert_string_coordinate": (c_int, [c_char_p, _P(c_double)]),
    "rt_light_position_from_square": (c_int, [c_char_p, _P(c_double)]),
    "rt_load_scene": (c_int, [_P(c_char_p), _P(c_int32), c_int, _P(rt_scene), _P(rt_sphere), c_int, _P(rt_mesh),
                              c_int, _P(rt_light)]),
    "rt_camera_init_reference": (c_int, [_P(rt_camera), c_int, c_int, c_double]),
    "rt_local_rows": (c_int, [c_int, _P(rt_rows), _P(c_int)]),
    "rt_global_row": (c_int, [c_int, _P(rt_rows), c_int, _P(c_int)]),
    "rt_set_scene": (c_int, [c_void_p, _P(rt_scene)]),
    "rt_render_dev": (c_int, [c_void_p, _P(rt_camera), c_int, c_int, c_int, _P(rt_rows), c_void_p, c_void_p,
                              c_void_p, c_void_p, c_void_p]),
    "rt_render": (c_int, [c_void_p, _P(rt_scene), _P(rt_camera), c_int, c_int, c_int, _P(rt_rows), c_void_p,
                          c_void_p, c_void_p, _P(rt_stats)]),
    "rt_intersect_dev": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p]),
    "rt_trace_rays_dev": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p]),
    "rt_unshuffle_dev": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p]),
    "rt_write_ppm": (c_int, [c_char_p, _P(c_uint8), c_int, c_int, c_int]),
    "rt_render_screen": (c_int, [c_void_p, _P(rt_scene), _P(rt_camera), c_int, c_int, c_int, c_int, ctypes.c_uint32,
                                 c_void_p, c_void_p, c_void_p, _P(ctypes.c_uint64)]),
    "rt_band_plan": (c_int, [c_int, c_int, c_int, _P(c_int), _P(c_int)]),
    "rt_group_create": (c_int, [_P(c_void_p), c_int, c_int, _P(c_void_p)]),
    "rt_comm_unique_id": (c_int, [c_void_p]),
    "rt_group_create_rank": (c_int, [c_void_p, c_int, c_int, c_void_p, _P(c_void_p)]),
    "rt_group_destroy": (c_int, [c_void_p]),
    "rt_group_info": (c_int, [c_void_p, _P(c_int), _P(c_int), _P(c_int), _P(c_int)]),
    "rt_render_multi": (c_int, [c_void_p, _P(rt_camera), c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p,
                                c_void_p]),
    "rt_group_synchronize": (c_int, [c_void_p]),
    "rt_group_timing": (c_int, [c_void_p, c_int]),
    "rt_group_get_stats": (c_int, [c_void_p, _P(rt_group_stats)]),
    "rt_pixel_bytes": (c_int, [c_int, _P(c_int)]),
    "rt_scene_achromatic": (c_int, [_P(rt_scene), _P(c_int)]),
    "rt_render_dev_packed": (c_int, [c_void_p, _P(rt_camera), c_int, c_int, c_int, _P(rt_rows), c_int, c_void_p,
                                     c_int, c_void_p, c_void_p]),
    "rt_render_packed": (c_int, [c_void_p, _P(rt_scene), _P(rt_camera), c_int, c_int, c_int, c_int, c_void_p,
                                 _P(rt_stats)]),
    "rt_render_packed_async": (c_int, [c_void_p, _P(rt_scene), _P(rt_camera), c_int, c_int, c_int, c_int, c_void_p,
                                       _P(c_uint64)]),
    "rt_ctx_wait": (c_int, [c_void_p, c_uint64]),
    "rt_host_alloc": (c_int, [ctypes.c_size_t, _P(c_void_p)]),
    "rt_host_free": (c_int, [c_void_p]),
    "rt_unpack_dev": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p]),
    "rt_group_plan_frame": (c_int, [c_int, c_int, c_int, c_int, c_int, c_int, c_int, _P(rt_group_plan)]),
    "rt_group_plan_recv": (c_int, [_P(rt_group_plan), c_int, c_int, c_int, c_int, _P(c_uint64), _P(c_uint64)]),
    "rt_group_root_renders": (c_int, [c_int]),
    "rt_scene_fingerprint": (c_int, [_P(rt_scene), _P(c_uint64)]),
    # include/rt_diag.h
    "rt_group_agree_due": (c_int, [c_uint64, c_int, c_uint64]),
    "rt_group_agree_vote": (None, [c_uint64, c_int, _P(c_uint64)]),
    "rt_group_agree_combine": (None, [_P(c_uint64), _P(c_uint64)]),
    "rt_group_agree_verdict": (c_int, [_P(c_uint64)]),
    "rt_probe_math_dev": (c_int, [c_int, c_void_p, c_int, c_void_p, c_void_p]),
    "rt_diag_tile_order": (c_int, [c_void_p, c_int]),
    "rt_diag_kernel_resources": (c_int, [c_int, c_int, _P(c_int), _P(c_int)]),
    "rt_diag_kernel_occupancy": (c_int, [c_int, c_int, c_int, _P(c_int)]),
    "rt_diag_copy_path": (c_int, [c_void_p, _P(c_int), _P(c_int)]),
}

_DIAG = {"rt_diag_tile_order", "rt_diag_kernel_resources", "rt_diag_kernel_occupancy", "rt_diag_copy_path"}
_lib = None


def lib() -> ctypes.CDLL:
    """Load ray_tracer_fragment_shader_amd/lib/librt_amd.so (built by __graft_entry__.build())."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; "
                               f"g.build()'` (make -C ray_tracer_fragment_shader_amd/csrc)")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            if name in _DIAG and not hasattr(L, name):
                continue                     # diagnostics of rt_diag.h (older builds in A/B timing tools)
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        if L.rt_abi_version() != ABI_VERSION:
            raise RuntimeError("librt_amd.so ABI version mismatch")
        _lib = L
    return _lib


def last_error() -> str:
    msg = lib().rt_last_error()
    return msg.decode() if msg else ""


def check(code: int, where: str) -> int:
    if code != RT_OK:
        raise RtError(code, where, last_error())
    return code


def vec3(v) -> "D3":
    return D3(*[float(x) for x in v])
