"""Device-side host wrapper over the C ABI (include/rt_api.h).

PyTorch is plumbing only: it owns HBM buffers and streams; every pixel is computed by the HIP kernels in
lib/librt_amd.so.  There is no fallback path — a missing library or device raises.
"""
from __future__ import annotations

import ctypes
from typing import Optional

import torch

from . import abi, scenes


def _ptr(t: Optional[torch.Tensor]):
    if t is None:
        return None
    if not t.is_cuda or not t.is_contiguous():
        raise ValueError("device buffers must be contiguous HIP tensors")
    return ctypes.c_void_p(t.data_ptr())


class Tracer:
    """One rt_ctx on one device (rt_ctx_create) holding the uploaded scene (rt_set_scene)."""

    def __init__(self, device: int = 0):
        self.device = device
        self._ctx = ctypes.c_void_p()
        abi.check(abi.lib().rt_ctx_create(device, ctypes.byref(self._ctx)), "rt_ctx_create")
        self._scene = None

    def close(self):
        if self._ctx:
            abi.lib().rt_ctx_destroy(self._ctx)
            self._ctx = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------------------------------------ scene
    def set_scene(self, scene: "scenes.Scene | abi.rt_scene"):
        s = scene.to_abi() if isinstance(scene, scenes.Scene) else scene
        abi.check(abi.lib().rt_set_scene(self._ctx, ctypes.byref(s)), "rt_set_scene")
        self._scene = scene

    # ----------------------------------------------------------------------------------------- render
    def alloc(self, width: int, height: int, rows: Optional[abi.rt_rows] = None, rgba32f=True, rgba8=False,
              rgb64f=False, raycount=False):
        nl = scenes.local_rows(height, rows)
        dev = torch.device("cuda", self.device)
        return {
            "rgba32f": torch.empty((nl, width, 4), dtype=torch.float32, device=dev) if rgba32f else None,
            "rgba8": torch.empty((nl, width, 4), dtype=torch.uint8, device=dev) if rgba8 else None,
            "rgb64f": torch.empty((nl, width, 3), dtype=torch.float64, device=dev) if rgb64f else None,
            "raycount": torch.empty((nl, width), dtype=torch.int32, device=dev) if raycount else None,
        }

    def render_into(self, cam: abi.rt_camera, width: int, height: int, depth: int, bufs: dict,
                    rows: Optional[abi.rt_rows] = None, stream: Optional[torch.cuda.Stream] = None):
        """rt_render_dev: asynchronous on `stream` (default: torch's current stream)."""
        st = stream if stream is not None else torch.cuda.current_stream(self.device)
        abi.check(abi.lib().rt_render_dev(self._ctx, ctypes.byref(cam), width, height, depth,
                                          ctypes.byref(rows) if rows is not None else None,
                                          _ptr(bufs.get("rgba32f")), _ptr(bufs.get("rgba8")),
                                          _ptr(bufs.get("rgb64f")), _ptr(bufs.get("raycount")),
                                          ctypes.c_void_p(st.cuda_stream)), "rt_render_dev")
        return bufs

    def render(self, cam, width, height, depth, rows=None, rgba32f=True, rgba8=False, rgb64f=False,
               raycount=False, stream=None):
        bufs = self.alloc(width, height, rows, rgba32f, rgba8, rgb64f, raycount)
        return self.render_into(cam, width, height, depth, bufs, rows, stream)

    def render_packed(self, cam, width, height, depth, float_format=None, byte_format=None, rows=None,
                      stream=None):
        """rt_render_dev_packed: the float image in float_format (RT_PIXEL_RGBA32F / GRAY32F) and the byte
        image in byte_format (RT_PIXEL_RGBA8 / RGB8 / GRAY8), each None to skip.  Returns (float, byte)
        tensors of shape (rows, W, channels)."""
        nl = scenes.local_rows(height, rows)
        dev = torch.device("cuda", self.device)
        ch = {abi.RT_PIXEL_RGBA32F: 4, abi.RT_PIXEL_GRAY32F: 1, abi.RT_PIXEL_RGBA8: 4, abi.RT_PIXEL_RGB8: 3,
              abi.RT_PIXEL_GRAY8: 1}
        f = torch.empty((nl, width, ch[float_format]), dtype=torch.float32, device=dev) if float_format is not None \
            else None
        b = torch.empty((nl, width, ch[byte_format]), dtype=torch.uint8, device=dev) if byte_format is not None \
            else None
        st = stream if stream is not None else torch.cuda.current_stream(self.device)
        abi.check(abi.lib().rt_render_dev_packed(
            self._ctx, ctypes.byref(cam), width, height, depth, ctypes.byref(rows) if rows is not None else None,
            float_format if float_format is not None else abi.RT_PIXEL_RGBA32F, _ptr(f),
            byte_format if byte_format is not None else abi.RT_PIXEL_RGBA8, _ptr(b),
            ctypes.c_void_p(st.cuda_stream)), "rt_render_dev_packed")
        return f, b

    def render_host(self, scene_abi, cam, width, height, depth, rows=None):
        """rt_render (host buffers, synchronous) -> (rgb64f numpy, rt_stats)."""
        import numpy as np
        nl = scenes.local_rows(height, rows)
        rgb = np.zeros((nl, width, 3), np.float64)
        st = abi.rt_stats()
        abi.check(abi.lib().rt_render(self._ctx, ctypes.byref(scene_abi), ctypes.byref(cam), width, height, depth,
                                      ctypes.byref(rows) if rows is not None else None, None, None,
                                      ctypes.c_void_p(rgb.ctypes.data), ctypes.byref(st)), "rt_render")
        return rgb, st

    # ------------------------------------------------------------------------------------ ray lists
    def trace_rays(self, starts: torch.Tensor, ends: torch.Tensor, depth: int, stream=None):
        n = starts.shape[0]
        rgb = torch.empty((n, 3), dtype=torch.float64, device=starts.device)
        rc = torch.empty((n,), dtype=torch.int32, device=starts.device)
        st = stream if stream is not None else torch.cuda.current_stream(self.device)
        abi.check(abi.lib().rt_trace_rays_dev(self._ctx, _ptr(starts), _ptr(ends), n, depth, _ptr(rgb), _ptr(rc),
                                              ctypes.c_void_p(st.cuda_stream)), "rt_trace_rays_dev")
        return rgb, rc

    def intersect(self, starts: torch.Tensor, ends: torch.Tensor, stream=None):
        n = starts.shape[0]
        raw = torch.empty((n, ctypes.sizeof(abi.rt_hit)), dtype=torch.uint8, device=starts.device)
        st = stream if stream is not None else torch.cuda.current_stream(self.device)
        abi.check(abi.lib().rt_intersect_dev(self._ctx, _ptr(starts), _ptr(ends), n, _ptr(raw),
                                             ctypes.c_void_p(st.cuda_stream)), "rt_intersect_dev")
        return raw


def unshuffle(gathered: torch.Tensor, image: torch.Tensor, width: int, height: int, band_height: int,
              n_ranks: int, slab_rows: int, stream=None):
    """rt_unshuffle_dev: gathered [n_ranks, slab_rows, W, C] -> image [H, W, C] (same dtype)."""
    elem = gathered.element_size() * (gathered.shape[-1] if gathered.dim() == 4 else 1)
    st = stream if stream is not None else torch.cuda.current_stream(image.device)
    abi.check(abi.lib().rt_unshuffle_dev(_ptr(gathered), _ptr(image), width, height, elem, band_height, n_ranks,
                                         slab_rows, ctypes.c_void_p(st.cuda_stream)), "rt_unshuffle_dev")
    return image


def unpack(gathered: torch.Tensor, image: torch.Tensor, width: int, height: int, src_format: int, dst_format: int,
           band_height: int, n_ranks: int, slab_rows: int, stream=None):
    """rt_unpack_dev: packed slabs (src_format) -> image (dst_format), bands put in image order."""
    st = stream if stream is not None else torch.cuda.current_stream(image.device)
    abi.check(abi.lib().rt_unpack_dev(_ptr(gathered), _ptr(image), width, height, src_format, dst_format, band_height,
                                      n_ranks, slab_rows, ctypes.c_void_p(st.cuda_stream)), "rt_unpack_dev")
    return image


def decode_hits(raw: torch.Tensor) -> dict:
    """rt_hit records (bytes) -> dict of numpy arrays (host)."""
    import numpy as np
    a = raw.cpu().numpy()
    n = a.shape[0]
    d = a[:, :96].copy().view(np.float64).reshape(n, 12)
    i = a[:, 96:104].copy().view(np.int32).reshape(n, 2)
    return {"point": d[:, 0:3], "normal": d[:, 3:6], "reflected_end": d[:, 6:9], "transmitted_end": d[:, 9:12],
            "hit": i[:, 0], "material": i[:, 1]}
