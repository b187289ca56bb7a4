"""GPU tests of the packed pixel formats (include/rt_api.h RT_PIXEL_*): the GRAY / RGB images the kernel writes
for the multi-GPU gather (rt_render_multi's wire formats) and for host frames (rt_render_packed, draw()'s
replacement with fewer PCIe bytes), their expansion (rt_unpack_dev), the group's per-phase timing, and the
bounding-sphere shortcut for rays from far origins.

The reference has one colour path (rayTraceRay, MySdlApplication.cpp:1184-1249); a packed image is exact when it
expands to the very bytes of the RGBA images a plain render writes — every test below checks that byte for byte,
and the RGBA images themselves are pinned to the reference elsewhere (test_gpu_parity.py)."""
import ctypes
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")

from oracle import pyoracle as po  # noqa: E402
from ray_tracer_fragment_shader_amd import abi, scenes  # noqa: E402
from ray_tracer_fragment_shader_amd.distributed import BandPlan  # noqa: E402
from ray_tracer_fragment_shader_amd.tracer import Tracer, unpack  # noqa: E402

from . import golden  # noqa: E402

pytestmark = pytest.mark.gpu
P = abi


@pytest.fixture(scope="module")
def tr():
    if not torch.cuda.is_available():
        pytest.fail("gpu tests need a HIP device")
    t = Tracer(0)
    yield t
    t.close()


def _chromatic_demo():
    """The app's demo board (MSA:1387-1428) — its cube material is red (MSA:588): not achromatic."""
    return scenes.load_scene([("b6", scenes.LIGHT), ("b4", scenes.TETRAHEDRON), ("d7", scenes.SPHERE),
                              ("a7", scenes.CUBE)])


def _rgba(tr, cam, W, H, depth, rows=None):
    b = tr.render(cam, W, H, depth, rows=rows, rgba32f=True, rgba8=True)
    torch.cuda.synchronize()
    return b["rgba32f"], b["rgba8"]


@pytest.mark.parametrize("name,W,H", [("c2", 480, 270), ("c3", 333, 187), ("c5", 640, 360), ("c1", 7, 5)])
def test_gray_formats_are_the_rgba_images(tr, name, W, H):
    """Achromatic scenes: R = G = B bit for bit, and GRAY32F / GRAY8 are exactly the R channel of RGBA32F / RGBA8;
    RGB8 is RGBA8 without alpha.  Also per band (rt_rows) and with both images in one launch."""
    cfg = scenes.CONFIGS[name]
    tr.set_scene(cfg.scene())
    cam = cfg.camera(W, H)
    f4, b4 = _rgba(tr, cam, W, H, cfg.depth)
    assert torch.equal(f4[..., 0], f4[..., 1]) and torch.equal(f4[..., 0], f4[..., 2])
    assert torch.equal(b4[..., 0], b4[..., 1]) and torch.equal(b4[..., 0], b4[..., 2])
    g32, g8 = tr.render_packed(cam, W, H, cfg.depth, P.RT_PIXEL_GRAY32F, P.RT_PIXEL_GRAY8)
    _, rgb8 = tr.render_packed(cam, W, H, cfg.depth, None, P.RT_PIXEL_RGB8)
    torch.cuda.synchronize()
    assert torch.equal(g32[..., 0], f4[..., 0])
    assert torch.equal(g8[..., 0], b4[..., 0])
    assert torch.equal(rgb8, b4[..., :3])
    rows = scenes.rows(3, 4, 2)
    f4r, b4r = _rgba(tr, cam, W, H, cfg.depth, rows=rows)
    g32r, g8r = tr.render_packed(cam, W, H, cfg.depth, P.RT_PIXEL_GRAY32F, P.RT_PIXEL_GRAY8, rows=rows)
    torch.cuda.synchronize()
    assert torch.equal(g32r[..., 0], f4r[..., 0]) and torch.equal(g8r[..., 0], b4r[..., 0])


def test_chromatic_scene_rejects_gray_and_packs_rgb(tr):
    sc = _chromatic_demo()
    tr.set_scene(sc)
    W, H = 200, 200
    cam = scenes.make_camera(W, H, 2.5)
    f4, b4 = _rgba(tr, cam, W, H, 5)
    assert not torch.equal(b4[..., 0], b4[..., 1])                  # the red cube shows
    _, rgb8 = tr.render_packed(cam, W, H, 5, None, P.RT_PIXEL_RGB8)
    torch.cuda.synchronize()
    assert torch.equal(rgb8, b4[..., :3])
    with pytest.raises(abi.RtError) as e:
        tr.render_packed(cam, W, H, 5, None, P.RT_PIXEL_GRAY8)
    assert e.value.code == abi.RT_EINVAL and "achromatic" in str(e.value)
    with pytest.raises(abi.RtError):
        tr.render_packed(cam, W, H, 5, P.RT_PIXEL_GRAY32F, None)
    with pytest.raises(abi.RtError):                                 # a byte format for the float image
        tr.render_packed(cam, W, H, 5, P.RT_PIXEL_RGB8, None)


# W % 4 == 0: unrolled 4-pixel steps (4352: more than one unrolled step per lane), else per pixel
@pytest.mark.parametrize("W", [480, 4352, 484, 477])
@pytest.mark.parametrize("G,hb", [(1, 0), (3, 5), (8, 0)])
def test_unpack_dev_expands_bands(tr, W, G, hb):
    """rt_unpack_dev: G ranks' packed bands -> RGBA images in image order, equal to the one-launch images."""
    cfg = scenes.CONFIGS["c3"]
    H = 270
    tr.set_scene(cfg.scene())
    cam = cfg.camera(W, H)
    f4, b4 = _rgba(tr, cam, W, H, cfg.depth)
    plan = BandPlan(H, G, hb)
    dev = "cuda"
    gath = {P.RT_PIXEL_GRAY32F: torch.zeros((G, plan.slab_rows, W), dtype=torch.float32, device=dev),
            P.RT_PIXEL_GRAY8: torch.zeros((G, plan.slab_rows, W), dtype=torch.uint8, device=dev),
            P.RT_PIXEL_RGB8: torch.zeros((G, plan.slab_rows, W, 3), dtype=torch.uint8, device=dev)}
    for r in range(G):
        n = plan.frame_local[r]
        g32, g8 = tr.render_packed(cam, W, H, cfg.depth, P.RT_PIXEL_GRAY32F, P.RT_PIXEL_GRAY8, rows=plan.rows(r))
        _, rgb = tr.render_packed(cam, W, H, cfg.depth, None, P.RT_PIXEL_RGB8, rows=plan.rows(r))
        gath[P.RT_PIXEL_GRAY32F][r, :n] = g32[..., 0]
        gath[P.RT_PIXEL_GRAY8][r, :n] = g8[..., 0]
        gath[P.RT_PIXEL_RGB8][r, :n] = rgb
    for src, dst, want in ((P.RT_PIXEL_GRAY32F, P.RT_PIXEL_RGBA32F, f4), (P.RT_PIXEL_GRAY8, P.RT_PIXEL_RGBA8, b4),
                           (P.RT_PIXEL_RGB8, P.RT_PIXEL_RGBA8, b4)):
        img = torch.full_like(want, 7)
        unpack(gath[src], img, W, H, src, dst, plan.band_height, G, plan.slab_rows)
        torch.cuda.synchronize()
        assert torch.equal(img, want), (src, dst)
    with pytest.raises(abi.RtError):                                 # no such expansion
        unpack(gath[P.RT_PIXEL_GRAY8], torch.empty_like(f4), W, H, P.RT_PIXEL_GRAY8, P.RT_PIXEL_RGBA32F,
               plan.band_height, G, plan.slab_rows)


def _group(ctxs, transport):
    arr = (ctypes.c_void_p * len(ctxs))(*[c._ctx.value for c in ctxs])
    g = ctypes.c_void_p()
    abi.check(abi.lib().rt_group_create(arr, len(ctxs), transport, ctypes.byref(g)), "rt_group_create")
    return g


def _multi(g, cam, W, H, depth, o32, o8, stream):
    outs = (P.RT_OUT_RGBA32F if o32 is not None else 0) | (P.RT_OUT_RGBA8 if o8 is not None else 0)
    abi.check(abi.lib().rt_render_multi(g, ctypes.byref(cam), W, H, depth, 0, outs,
                                        ctypes.c_void_p(o32.data_ptr()) if o32 is not None else None,
                                        ctypes.c_void_p(o8.data_ptr()) if o8 is not None else None,
                                        ctypes.c_void_p(stream.cuda_stream)), "rt_render_multi")


def _stats(g):
    st = abi.rt_group_stats()
    abi.check(abi.lib().rt_group_get_stats(g, ctypes.byref(st)), "rt_group_get_stats")
    return st


@pytest.mark.parametrize("kind", ["achromatic", "chromatic"])
@pytest.mark.parametrize("n", [2, 4])
def test_render_multi_wire_formats(tr, kind, n):
    """rt_render_multi sends GRAY8 / GRAY32F for an achromatic scene and RGB8 / RGBA32F otherwise; rank 0's
    images equal one launch's byte for byte (several frames, alternating eyes, double buffers in flight), and
    the per-phase timing and payload match the wire formats."""
    if kind == "achromatic":
        cfg = scenes.CONFIGS["c3"]
        sc, W, H, depth = cfg.scene(), 1280, 720, cfg.depth
        cams = [cfg.camera(W, H), cfg.camera(W, H)]
    else:
        sc, W, H, depth = _chromatic_demo(), 500, 500, 5
        cams = [scenes.make_camera(W, H, 1.0), scenes.make_camera(W, H, 1.0)]
    cams[1].eye = abi.vec3((30.0, 140.0, 260.0))
    ctxs = [Tracer(0) for _ in range(n)]
    for c in ctxs:
        c.set_scene(sc)
    g = _group(ctxs, P.RT_TRANSPORT_COPY)
    try:
        tr.set_scene(sc)
        want = [tuple(x.clone() for x in _rgba(tr, c, W, H, depth)) for c in cams]
        s = torch.cuda.Stream()
        abi.check(abi.lib().rt_group_timing(g, 1), "rt_group_timing")
        outs = [(torch.empty((H, W, 4), dtype=torch.float32, device="cuda"),
                 torch.empty((H, W, 4), dtype=torch.uint8, device="cuda")) for _ in range(6)]
        for f in range(6):
            _multi(g, cams[f % 2], W, H, depth, outs[f][0], outs[f][1], s)
        s.synchronize()
        for f in range(6):
            assert torch.equal(outs[f][0], want[f % 2][0]), f"frame {f} RGBA32F differs"
            assert torch.equal(outs[f][1], want[f % 2][1]), f"frame {f} RGBA8 differs"
        st = _stats(g)
        achro = kind == "achromatic"
        assert st.frames == 6 and st.ranks_timed == n
        assert st.wire_float == (P.RT_PIXEL_GRAY32F if achro else P.RT_PIXEL_RGBA32F)
        assert st.wire_byte == (P.RT_PIXEL_GRAY8 if achro else P.RT_PIXEL_RGB8)
        per_px = (4 + 1) if achro else (16 + 3)
        if abi.lib().rt_group_root_renders(n):              # rank 0's own bands stay local
            assert st.payload_bytes == sum(BandPlan(H, n).frame_local[1:]) * W * per_px
        else:                                                 # rank 0 only assembles: every row arrives
            assert st.payload_bytes == H * W * per_px
        assert st.render_ms > 0 and st.gather_ms > 0 and st.assemble_ms > 0
        assert st.frame_ms >= st.render_ms
        # the byte image alone (what the bench gathers)
        o8 = torch.empty((H, W, 4), dtype=torch.uint8, device="cuda")
        _multi(g, cams[0], W, H, depth, None, o8, s)
        s.synchronize()
        assert torch.equal(o8, want[0][1])
        assert _stats(g).wire_float == -1
    finally:
        abi.lib().rt_group_destroy(g)
        for c in ctxs:
            c.close()


def test_render_multi_regrow_when_width_changes(tr):
    """Buffers that must grow (a wider frame with the same band plan) wait for the frames still using them."""
    cfg = scenes.CONFIGS["c2"]
    sc = cfg.scene()
    ctxs = [Tracer(0) for _ in range(3)]
    for c in ctxs:
        c.set_scene(sc)
    g = _group(ctxs, P.RT_TRANSPORT_COPY)
    try:
        tr.set_scene(sc)
        s = torch.cuda.Stream()
        H = 240
        frames = []
        for W in (320, 320, 960, 320, 1280):
            o8 = torch.empty((H, W, 4), dtype=torch.uint8, device="cuda")
            _multi(g, cfg.camera(W, H), W, H, cfg.depth, None, o8, s)
            frames.append((W, o8))
        s.synchronize()
        for W, o8 in frames:
            assert torch.equal(o8, _rgba(tr, cfg.camera(W, H), W, H, cfg.depth)[1]), W
    finally:
        abi.lib().rt_group_destroy(g)
        for c in ctxs:
            c.close()


def test_render_multi_c5_full_size_8_ranks_hash(tr):
    """c5 as BASELINE names it (7680x4320, 64 spheres, 3 bounces, split over 8 ranks): rt_render_multi with 8
    ranks (device-copy transport on one GPU; the RCCL transport moves the same slabs) — the assembled RGBA32F
    frame is the float rounding of the one-launch float64 frame, which hashes to the reference's own c5 frame."""
    cfg = scenes.CONFIGS["c5"]
    W, H = cfg.width, cfg.height
    sc = cfg.scene()
    ctxs = [Tracer(0) for _ in range(8)]
    for c in ctxs:
        c.set_scene(sc)
    g = _group(ctxs, P.RT_TRANSPORT_AUTO)
    try:
        s = torch.cuda.Stream()
        o32 = torch.empty((H, W, 4), dtype=torch.float32, device="cuda")
        o8 = torch.empty((H, W, 4), dtype=torch.uint8, device="cuda")
        _multi(g, cfg.camera(), W, H, cfg.depth, o32, o8, s)
        s.synchronize()
        tr.set_scene(sc)
        b = tr.render(cfg.camera(), W, H, cfg.depth, rgba32f=False, rgba8=True, rgb64f=True)
        torch.cuda.synchronize()
        rgb = b["rgb64f"].cpu().numpy()
        assert f"{po.fnv1a64(rgb):016x}" == golden.manifest()["frames"]["c5"]["fnv1a64"]
        assert np.array_equal(o32.cpu().numpy()[..., :3], rgb.astype(np.float32))
        assert torch.equal(o8, b["rgba8"])
        assert _stats(g).wire_byte == P.RT_PIXEL_GRAY8
    finally:
        abi.lib().rt_group_destroy(g)
        for c in ctxs:
            c.close()


def _host_alloc(nbytes):
    p = ctypes.c_void_p()
    abi.check(abi.lib().rt_host_alloc(nbytes, ctypes.byref(p)), "rt_host_alloc")
    return p


# the defaults (synchronous: copy kernel behind the render; pipelined: SDMA engine), the copy kernel for both (on the
# copy stream), the SDMA engine for both
COPY_MODES = [None, "0", "3"]
_SYNC_MODE = {None: 1, "0": 0, "3": 3}    # what rt_diag_copy_path reports after a synchronous pinned frame
_ASYNC_MODE = {None: 3, "0": 0, "3": 3}   # ... after a pipelined one


def _copy_path(t):
    mode, writer = ctypes.c_int(), ctypes.c_int()
    abi.check(abi.lib().rt_diag_copy_path(t._ctx, ctypes.byref(mode), ctypes.byref(writer)), "rt_diag_copy_path")
    return mode.value, writer.value


# The cases whose frames leave on the SDMA engines (HSA copies the HIP runtime does not schedule) run in ONE child
# process of their own, test_sdma_cases_in_child_process: the round's full GPU-suite runs stopped three times with an
# illegal address raised by a later device-to-host copy of the runtime's own, always after these cases had run in the
# same process.  In the pytest process they report "skipped: run in the SDMA child process".
_SDMA_CHILD = os.environ.get("RT_TEST_SDMA_CHILD") == "1"
_SDMA_CASES = [("test_render_packed_host_sync_and_async", {"copy_mode": None}),
               ("test_render_packed_host_sync_and_async", {"copy_mode": "3"}),
               ("test_render_packed_two_behind_and_mixed_sync", {"copy_mode": None}),
               ("test_render_packed_two_behind_and_mixed_sync", {"copy_mode": "3"}),
               ("test_render_packed_sdma_one_or_two_engines", {"split": "1"}),
               ("test_render_packed_sdma_one_or_two_engines", {"split": "2"}),
               ("test_render_packed_sdma_into_registered_memory", {}),
               ("test_render_packed_sdma_slow_render_is_not_a_failure", {"writer": "2"}),
               ("test_render_packed_sdma_slow_render_is_not_a_failure", {"writer": "1"})]


def _sdma_only_in_child():
    if not _SDMA_CHILD:
        pytest.skip("runs in the SDMA child process (test_sdma_cases_in_child_process)")


def test_sdma_cases_in_child_process():
    """Every SDMA case above, in one child process (a fresh HIP runtime), each with its own environment."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = ("import os, sys\n"
            "sys.path.insert(0, %r)\n"
            "os.environ['RT_TEST_SDMA_CHILD'] = '1'\n"
            "import pytest\n"
            "from _pytest.monkeypatch import MonkeyPatch\n"
            "from tests import test_gpu_packed as m\n"
            "from ray_tracer_fragment_shader_amd.tracer import Tracer\n"
            "tr = Tracer(0)\n"
            "for name, kw in m._SDMA_CASES:\n"
            "    mp = MonkeyPatch()\n"
            "    try:\n"
            "        getattr(m, name)(tr=tr, monkeypatch=mp, **kw)\n"
            "        print('ok', name, kw, flush=True)\n"
            "    except pytest.skip.Exception as e:\n"
            "        print('skipped', name, kw, e, flush=True)\n"
            "    finally:\n"
            "        mp.undo()\n"
            "tr.close()\n"
            "print('done', flush=True)\n") % root
    env = {k: v for k, v in os.environ.items() if not k.startswith("RT_")}
    r = subprocess.run([sys.executable, "-c", code], cwd=root, env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0 and r.stdout.strip().endswith("done"), (r.returncode, r.stdout[-3000:], r.stderr[-3000:])
    assert r.stdout.count("ok ") + r.stdout.count("skipped ") == len(_SDMA_CASES), r.stdout
    assert r.stdout.count("ok ") >= len(_SDMA_CASES) - 1, r.stdout      # (only the host-register case may skip)
    print(r.stdout)


@pytest.mark.parametrize("copy_mode", COPY_MODES, ids=["default", "copy_stream", "sdma"])
def test_render_packed_host_sync_and_async(tr, monkeypatch, copy_mode):
    """rt_render_packed (synchronous, pinned and pageable host buffers, stats) and rt_render_packed_async (a
    pipelined stream of frames with alternating eyes into two pinned buffers, each waited for by its ticket):
    every frame equals the device render's bytes — with the copy kernel and with the SDMA engine."""
    if copy_mode != "0":
        _sdma_only_in_child()
    if copy_mode:
        monkeypatch.setenv("RT_COPY_MODE", copy_mode)
    L = abi.lib()
    cfg = scenes.CONFIGS["c2"]
    sa = cfg.scene().to_abi()
    W, H = 960, 540
    cams = [cfg.camera(W, H), cfg.camera(W, H)]
    cams[1].eye = abi.vec3((-40.0, 120.0, 230.0))
    tr.set_scene(cfg.scene())
    want = [_rgba(tr, c, W, H, cfg.depth)[1].cpu().numpy() for c in cams]
    t = Tracer(0)
    pins = [_host_alloc(W * H * 4) for _ in range(2)]
    try:
        for fmt, ch in ((P.RT_PIXEL_GRAY8, 1), (P.RT_PIXEL_RGB8, 3), (P.RT_PIXEL_RGBA8, 4)):
            page = np.zeros((H, W, ch), np.uint8)
            st = abi.rt_stats()
            abi.check(L.rt_render_packed(t._ctx, ctypes.byref(sa), ctypes.byref(cams[0]), W, H, cfg.depth, fmt,
                                         ctypes.c_void_p(page.ctypes.data), ctypes.byref(st)), "rt_render_packed")
            assert np.array_equal(page, want[0][..., :ch] if ch > 1 else want[0][..., :1]), fmt
            assert st.primary_rays == W * H and st.kernel_ms > 0
            abi.check(L.rt_render_packed(t._ctx, ctypes.byref(sa), ctypes.byref(cams[1]), W, H, cfg.depth, fmt,
                                         pins[0], None), "rt_render_packed")
            got = np.ctypeslib.as_array(ctypes.cast(pins[0], ctypes.POINTER(ctypes.c_uint8)), (H, W, ch))
            assert np.array_equal(got, want[1][..., :ch]), fmt
            # a pinned buffer takes the requested engine (the pageable one above cannot)
            assert _copy_path(t)[0] == _SYNC_MODE[copy_mode], _copy_path(t)
        tickets = []
        for f in range(8):
            tk = ctypes.c_uint64()
            abi.check(L.rt_render_packed_async(t._ctx, ctypes.byref(sa), ctypes.byref(cams[f % 2]), W, H, cfg.depth,
                                               P.RT_PIXEL_GRAY8, pins[f % 2], ctypes.byref(tk)), "async")
            tickets.append(tk.value)
            if f >= 1:                                  # frame f-1 is complete once its ticket is waited for
                abi.check(L.rt_ctx_wait(t._ctx, tickets[f - 1]), "rt_ctx_wait")
                got = np.ctypeslib.as_array(ctypes.cast(pins[(f - 1) % 2], ctypes.POINTER(ctypes.c_uint8)), (H, W))
                assert np.array_equal(got, want[(f - 1) % 2][..., 0]), f - 1
        assert tickets == sorted(tickets) and len(set(tickets)) == 8
        assert _copy_path(t) == (_ASYNC_MODE[copy_mode], 2 if _ASYNC_MODE[copy_mode] == 3 else _copy_path(t)[1])
        abi.check(L.rt_ctx_wait(t._ctx, 0), "rt_ctx_wait")
        assert L.rt_ctx_wait(t._ctx, tickets[-1] + 5) == abi.RT_EINVAL
    finally:
        for p in pins:
            L.rt_host_free(p)
        t.close()


@pytest.mark.parametrize("copy_mode", COPY_MODES, ids=["default", "copy_stream", "sdma"])
def test_render_packed_two_behind_and_mixed_sync(tr, monkeypatch, copy_mode):
    """rt_render_packed_async with two frames waited for behind the one being queued (three pinned buffers, the
    copies on the copy stream or the SDMA engine), interleaved with synchronous rt_render_packed calls that reuse the
    same device slots: every frame, waited for by its ticket, equals the device render."""
    if copy_mode != "0":
        _sdma_only_in_child()
    if copy_mode:
        monkeypatch.setenv("RT_COPY_MODE", copy_mode)
    L = abi.lib()
    cfg = scenes.CONFIGS["c2"]
    sa = cfg.scene().to_abi()
    W, H = 640, 360
    cams = [cfg.camera(W, H) for _ in range(3)]
    cams[1].eye = abi.vec3((-40.0, 120.0, 230.0))
    cams[2].eye = abi.vec3((35.0, 90.0, 210.0))
    tr.set_scene(cfg.scene())
    want = [_rgba(tr, c, W, H, cfg.depth)[1].cpu().numpy()[..., 0] for c in cams]
    t = Tracer(0)
    pins = [_host_alloc(W * H) for _ in range(4)]
    try:
        tickets = []
        for f in range(12):
            tk = ctypes.c_uint64()
            abi.check(L.rt_render_packed_async(t._ctx, ctypes.byref(sa), ctypes.byref(cams[f % 3]), W, H, cfg.depth,
                                               P.RT_PIXEL_GRAY8, pins[f % 3], ctypes.byref(tk)), "async")
            tickets.append(tk.value)
            if f % 4 == 3:                               # a synchronous frame in between (render-stream copy)
                abi.check(L.rt_render_packed(t._ctx, ctypes.byref(sa), ctypes.byref(cams[(f + 1) % 3]), W, H,
                                             cfg.depth, P.RT_PIXEL_GRAY8, pins[3], None), "rt_render_packed")
                got = np.ctypeslib.as_array(ctypes.cast(pins[3], ctypes.POINTER(ctypes.c_uint8)), (H, W))
                assert np.array_equal(got, want[(f + 1) % 3]), f"sync after {f}"
            if f >= 2:
                abi.check(L.rt_ctx_wait(t._ctx, tickets[f - 2]), "rt_ctx_wait")
                got = np.ctypeslib.as_array(ctypes.cast(pins[(f - 2) % 3], ctypes.POINTER(ctypes.c_uint8)), (H, W))
                assert np.array_equal(got, want[(f - 2) % 3]), f - 2
        abi.check(L.rt_ctx_wait(t._ctx, 0), "rt_ctx_wait")
        assert _copy_path(t)[0] == _SYNC_MODE[copy_mode], _copy_path(t)   # the last frame was synchronous
        for f in (10, 11):
            got = np.ctypeslib.as_array(ctypes.cast(pins[f % 3], ctypes.POINTER(ctypes.c_uint8)), (H, W))
            assert np.array_equal(got, want[f % 3]), f
    finally:
        for p in pins:
            L.rt_host_free(p)
        t.close()


@pytest.mark.parametrize("split", ["1", "2"])
def test_render_packed_sdma_one_or_two_engines(tr, monkeypatch, split):
    """The SDMA path with the frame copied whole by one engine (RT_SDMA_SPLIT=1, or a frame under 64 KiB) or in
    halves by two: synchronous and pipelined frames equal the device render, byte for byte."""
    _sdma_only_in_child()
    monkeypatch.setenv("RT_COPY_MODE", "3")
    monkeypatch.setenv("RT_SDMA_SPLIT", split)
    L = abi.lib()
    cfg = scenes.CONFIGS["c2"]
    sa = cfg.scene().to_abi()
    tr.set_scene(cfg.scene())
    t = Tracer(0)
    try:
        for W, H in ((64, 48), (640, 360)):              # 3 KB (one piece whatever the split) and 230 KB
            cam = cfg.camera(W, H)
            want = _rgba(tr, cam, W, H, cfg.depth)[1].cpu().numpy()[..., 0]
            pins = [_host_alloc(W * H) for _ in range(3)]
            try:
                abi.check(L.rt_render_packed(t._ctx, ctypes.byref(sa), ctypes.byref(cam), W, H, cfg.depth,
                                             P.RT_PIXEL_GRAY8, pins[0], None), "rt_render_packed")
                assert _copy_path(t)[0] == 3
                got = np.ctypeslib.as_array(ctypes.cast(pins[0], ctypes.POINTER(ctypes.c_uint8)), (H, W))
                assert np.array_equal(got, want), (W, H)
                tk = [ctypes.c_uint64() for _ in range(3)]
                for f in range(6):
                    abi.check(L.rt_render_packed_async(t._ctx, ctypes.byref(sa), ctypes.byref(cam), W, H, cfg.depth,
                                                       P.RT_PIXEL_GRAY8, pins[f % 3], ctypes.byref(tk[f % 3])), "async")
                abi.check(L.rt_ctx_wait(t._ctx, 0), "rt_ctx_wait")
                for j in range(3):
                    got = np.ctypeslib.as_array(ctypes.cast(pins[j], ctypes.POINTER(ctypes.c_uint8)), (H, W))
                    assert np.array_equal(got, want), (W, H, j)
            finally:
                for p in pins:
                    L.rt_host_free(p)
    finally:
        t.close()


def test_render_packed_sdma_into_registered_memory(tr, monkeypatch):
    """Host memory the caller page-locked after allocating it (hipHostRegister) is reached by the SDMA engines at its
    device-side address: synchronous and pipelined frames into it equal the device render."""
    _sdma_only_in_child()
    cudart = torch.cuda.cudart()
    if not hasattr(cudart, "cudaHostRegister"):
        pytest.skip("no host-register binding in this torch")
    monkeypatch.setenv("RT_COPY_MODE", "3")
    L = abi.lib()
    cfg = scenes.CONFIGS["c2"]
    sa = cfg.scene().to_abi()
    W, H = 640, 360
    cam = cfg.camera(W, H)
    tr.set_scene(cfg.scene())
    want = _rgba(tr, cam, W, H, cfg.depth)[1].cpu().numpy()[..., 0]
    bufs = [np.zeros((H, W), np.uint8) for _ in range(3)]
    for b in bufs:
        assert int(cudart.cudaHostRegister(b.ctypes.data, b.nbytes, 0)) == 0
    t = Tracer(0)
    try:
        abi.check(L.rt_render_packed(t._ctx, ctypes.byref(sa), ctypes.byref(cam), W, H, cfg.depth, P.RT_PIXEL_GRAY8,
                                     ctypes.c_void_p(bufs[0].ctypes.data), None), "rt_render_packed")
        assert _copy_path(t)[0] == 3
        assert np.array_equal(bufs[0], want)
        for b in bufs:
            b[:] = 0
        tk = [ctypes.c_uint64() for _ in range(3)]
        for f in range(6):
            abi.check(L.rt_render_packed_async(t._ctx, ctypes.byref(sa), ctypes.byref(cam), W, H, cfg.depth,
                                               P.RT_PIXEL_GRAY8, ctypes.c_void_p(bufs[f % 3].ctypes.data),
                                               ctypes.byref(tk[f % 3])), "async")
        abi.check(L.rt_ctx_wait(t._ctx, 0), "rt_ctx_wait")
        for b in bufs:
            assert np.array_equal(b, want)
    finally:
        t.close()
        for b in bufs:
            cudart.cudaHostUnregister(b.ctypes.data)


def test_hits_inside_shortcut_far_origins(tr):
    """Rays from hit points skip the bounding-sphere cull only when the host proved every hit point lies inside
    its shortcut radius with a slack that covers the hit point's rounding, which grows with the level-0 origin's
    distance: per ray (ray lists) and per camera eye (renders).  A sphere placed 0.5 units inside that radius,
    rays and eyes from 1e2 to 1e17 away: every colour and ray count equals the oracle's (which always tests)."""
    R1 = np.sqrt(3.0) * 160.0 - 1.0
    x, y, z = scenes.convert_string_coordinate("a1")
    dx, dz = x, z                                        # world = local + (0, 0, -160) = local + bound centre
    yoff = np.sqrt((R1 - 0.5 - 20.0) ** 2 - dx * dx - dz * dz) - y
    sc = scenes.Scene(spheres=[scenes.SphereSpec("a1", 20.0, float(yoff)), scenes.SphereSpec("d5", 20.0)],
                      lights=[scenes.LightSpec("b6", scenes.WHITE), scenes.LightSpec("g3", scenes.GREY)])
    tr.set_scene(sc)
    c = np.array(sc.spheres[0].center()) + np.array([0.0, 0.0, -160.0])
    rng = np.random.default_rng(3)
    n = 4096
    dist = np.repeat([1e2, 1e6, 1e8, 1e12, 1e16, 1e17], n // 6 + 1)[:n]
    dirs = rng.normal(size=(n, 3))
    dirs /= np.linalg.norm(dirs, axis=1, keepdims=True)
    dirs[:, 1] = np.abs(dirs[:, 1])                      # from above the board
    starts = c + dirs * dist[:, None]
    ends = c + rng.normal(size=(n, 3)) * 10.0
    S, E = torch.tensor(starts, device="cuda"), torch.tensor(ends, device="cuda")
    for depth in (1, 2):
        rgb, rc = tr.trace_rays(S, E, depth)
        want, want_rc = po.trace_rays(sc.to_abi(), starts, ends, depth)
        got = rgb.cpu().numpy()
        assert np.array_equal(got, want, equal_nan=True), depth
        assert np.array_equal(rc.cpu().numpy().view(np.uint32), want_rc), depth
    W, H = 96, 64
    for d in (1e3, 1e8, 1e16):
        cam = scenes.make_camera(W, H, 1.0)
        cam.eye = abi.vec3(tuple(c + np.array([0.3, 0.8, 0.5]) / np.linalg.norm([0.3, 0.8, 0.5]) * d))
        cam.look_at = abi.vec3(tuple(c))
        cam.pitch = 60.0 / W
        b = tr.render(cam, W, H, 2, rgba32f=False, rgb64f=True, raycount=True)
        torch.cuda.synchronize()
        want, want_rc = po.render(sc.to_abi(), cam, W, H, 2)
        assert np.array_equal(b["rgb64f"].cpu().numpy(), want, equal_nan=True), d
        assert np.array_equal(b["raycount"].cpu().numpy().view(np.uint32), want_rc), d


@pytest.mark.parametrize("offset", [0, 16, 3])
def test_host_frames_into_pinned_interior_pointers(tr, offset):
    """Host frames land in rt_host_alloc memory through the device copy kernel (16-byte aligned) or
    hipMemcpyAsync (unaligned), also at an offset inside the allocation; rt_render's RGBA8 and rt_render_packed's
    GRAY8 equal the device render either way."""
    L = abi.lib()
    cfg = scenes.CONFIGS["c2"]
    sa = cfg.scene().to_abi()
    W, H = 333, 201
    cam = cfg.camera(W, H)
    tr.set_scene(cfg.scene())
    want = _rgba(tr, cam, W, H, cfg.depth)[1].cpu().numpy()
    t = Tracer(0)
    base = _host_alloc(W * H * 4 + 64)
    try:
        ptr = ctypes.c_void_p(base.value + offset)
        abi.check(L.rt_render(t._ctx, ctypes.byref(sa), ctypes.byref(cam), W, H, cfg.depth, None, None, ptr, None,
                              None), "rt_render")
        got = np.ctypeslib.as_array(ctypes.cast(ptr, ctypes.POINTER(ctypes.c_uint8)), (H, W, 4)).copy()
        assert np.array_equal(got, want)
        abi.check(L.rt_render_packed(t._ctx, ctypes.byref(sa), ctypes.byref(cam), W, H, cfg.depth, P.RT_PIXEL_GRAY8,
                                     ptr, None), "rt_render_packed")
        got = np.ctypeslib.as_array(ctypes.cast(ptr, ctypes.POINTER(ctypes.c_uint8)), (H, W)).copy()
        assert np.array_equal(got, want[..., 0])
    finally:
        L.rt_host_free(base)
        t.close()


def _slow_render_frames(tr, writer):
    """The body of test_render_packed_sdma_slow_render_is_not_a_failure (RT_COPY_MODE=3, RT_SDMA_WAIT_MS=0 and
    RT_SDMA_WRITER=writer already in the environment); also run as a child process for writer 1."""
    L = abi.lib()
    cfg = scenes.CONFIGS["c3"]
    sa = cfg.scene().to_abi()
    W, H = 1920, 1080
    cams = [cfg.camera(W, H) for _ in range(3)]
    cams[1].eye = abi.vec3((-40.0, 120.0, 230.0))
    cams[2].eye = abi.vec3((35.0, 90.0, 210.0))
    tr.set_scene(cfg.scene())
    want = [_rgba(tr, c, W, H, cfg.depth)[1].cpu().numpy()[..., 0] for c in cams]
    t = Tracer(0)
    pins = [_host_alloc(W * H) for _ in range(3)]
    try:
        tickets = []
        for f in range(12):
            tk = ctypes.c_uint64()
            abi.check(L.rt_render_packed_async(t._ctx, ctypes.byref(sa), ctypes.byref(cams[f % 3]), W, H, cfg.depth,
                                               P.RT_PIXEL_GRAY8, pins[f % 3], ctypes.byref(tk)), "async")
            tickets.append(tk.value)
            if f >= 2:
                abi.check(L.rt_ctx_wait(t._ctx, tickets[f - 2]), "rt_ctx_wait")
                got = np.ctypeslib.as_array(ctypes.cast(pins[(f - 2) % 3], ctypes.POINTER(ctypes.c_uint8)), (H, W))
                assert np.array_equal(got, want[(f - 2) % 3]), f - 2
        assert _copy_path(t) == (3, int(writer))
        abi.check(L.rt_ctx_wait(t._ctx, 0), "rt_ctx_wait")
        for f in (10, 11):
            got = np.ctypeslib.as_array(ctypes.cast(pins[f % 3], ctypes.POINTER(ctypes.c_uint8)), (H, W))
            assert np.array_equal(got, want[f % 3]), f
        abi.check(L.rt_render_packed(t._ctx, ctypes.byref(sa), ctypes.byref(cams[1]), W, H, cfg.depth,
                                     P.RT_PIXEL_GRAY8, pins[0], None), "rt_render_packed")
        got = np.ctypeslib.as_array(ctypes.cast(pins[0], ctypes.POINTER(ctypes.c_uint8)), (H, W))
        assert np.array_equal(got, want[1])
    finally:
        for p in pins:
            L.rt_host_free(p)
        t.close()


@pytest.mark.parametrize("writer", ["1", "2"])
def test_render_packed_sdma_slow_render_is_not_a_failure(tr, monkeypatch, writer):
    """sdma_wait's progress check at RT_SDMA_WAIT_MS=0 (every wait passes its deadline at once): a render still
    running when the deadline passes is waited for, not released by hand, so no copy starts before its frame is in its
    buffer — pipelined frames two behind, alternating views, each equal to the device render.  Both writers of the
    render stream's dependency store (RT_SDMA_WRITER): the signal kernel (the default) and the stream's write-value
    operation."""
    _sdma_only_in_child()
    monkeypatch.setenv("RT_COPY_MODE", "3")
    monkeypatch.setenv("RT_SDMA_WAIT_MS", "0")
    monkeypatch.setenv("RT_SDMA_WRITER", writer)
    _slow_render_frames(tr, writer)
