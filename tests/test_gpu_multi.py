"""GPU tests of the multi-GPU path (BASELINE config c4), the C++ drop-in
and the context's stream / graph / caching rules (rt_api.h).

c4 is c3 (3840x2160, 8 spheres + board, 2 lights, 2 bounces) with its rows split over 8 GPUs and gathered to
one.  A one-GPU box cannot hold 8 RCCL ranks (RCCL refuses two ranks on one device), so:
  * the row split itself is checked at full c4 size with n ranks' bands rendered on the one GPU, gathered and
    put in image order with rt_unshuffle_dev: the assembled float64 frame must hash to the reference's own c3
    frame (tests/golden/manifest.json) and the ray total must equal the reference's 18,956,255;
  * rt_render_multi (the C-ABI group) runs with n contexts sharing the GPU (device-copy transport: the same
    bands, slabs, double buffers, events and assembly as the RCCL transport) and with one context over RCCL
    (a one-rank communicator: ncclSend/ncclRecv to self through the same group calls).
"""
import ctypes
import os
import subprocess

import numpy as np
import pytest

torch = pytest.importorskip("torch")

from oracle import pyoracle as po  # noqa: E402
from ray_tracer_fragment_shader_amd import abi, scenes  # noqa: E402
from ray_tracer_fragment_shader_amd.distributed import BandPlan  # noqa: E402
from ray_tracer_fragment_shader_amd.tracer import Tracer, unshuffle  # noqa: E402

from . import golden  # noqa: E402

pytestmark = pytest.mark.gpu
LIBDIR = os.path.dirname(abi.LIB_PATH)


@pytest.fixture(scope="module")
def tr():
    if not torch.cuda.is_available():
        pytest.fail("gpu tests need a HIP device")
    t = Tracer(0)
    yield t
    t.close()


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


@pytest.mark.parametrize("n", [2, 4, 8])
def test_c4_row_split_full_size_vs_reference_hash(tr, n):
    """c4 geometry at full size: n ranks' round-robin bands (auto band height: the 8-row tile height, 34 / 33 bands
    per rank at n = 8), each rendered as its own launch, gathered into padded slabs and unshuffled on the device."""
    cfg = scenes.CONFIGS["c3"]
    W, H = cfg.width, cfg.height
    plan = BandPlan(H, n)
    if n == 8:
        assert plan.band_height == 8 and max(plan.frame_local) == 272 and min(plan.frame_local) == 264
    tr.set_scene(cfg.scene())
    cam = cfg.camera()
    gathered = torch.zeros((n, plan.slab_rows, W, 3), dtype=torch.float64, device="cuda")
    rays = 0
    for r in range(n):
        b = tr.render(cam, W, H, cfg.depth, rows=plan.rows(r), rgba32f=False, rgb64f=True, raycount=True)
        gathered[r, : plan.frame_local[r]] = b["rgb64f"]
        rc = b["raycount"].view(torch.int32)
        rays += int((rc & 0xFFFF).sum().item()) + int((rc >> 16).sum().item())
    img = torch.empty((H, W, 3), dtype=torch.float64, device="cuda")
    unshuffle(gathered, img, W, H, plan.band_height, n, plan.slab_rows)
    torch.cuda.synchronize()
    assert f"{po.fnv1a64(img.cpu().numpy()):016x}" == golden.manifest()["frames"]["c3"]["fnv1a64"]
    assert rays == scenes.PINNED_RAYS["c3"]


def _group(ctxs, transport):
    arr = (ctypes.c_void_p * len(ctxs))(*[c._ctx.value for c in ctxs])
    g = ctypes.c_void_p()
    abi.check(abi.lib().rt_group_create(arr, len(ctxs), transport, ctypes.byref(g)), "rt_group_create")
    return g


def _multi(g, cam, W, H, depth, hb, o32, o8, stream):
    outs = (abi.RT_OUT_RGBA32F if o32 is not None else 0) | (abi.RT_OUT_RGBA8 if o8 is not None else 0)
    abi.check(abi.lib().rt_render_multi(g, ctypes.byref(cam), W, H, depth, hb, outs, _ptr(o32), _ptr(o8),
                                        ctypes.c_void_p(stream.cuda_stream)), "rt_render_multi")


@pytest.mark.parametrize("n,transport,hb", [(1, abi.RT_TRANSPORT_RCCL, 0), (1, abi.RT_TRANSPORT_COPY, 0),
                                            (2, abi.RT_TRANSPORT_AUTO, 0), (3, abi.RT_TRANSPORT_COPY, 5),
                                            (8, abi.RT_TRANSPORT_AUTO, 0)])
def test_render_multi_matches_single_gpu(tr, n, transport, hb):
    """rt_render_multi over n ranks equals the one-launch frame (RGBA32F and RGBA8, every byte), for several
    frames in a row with alternating eyes (the double-buffered slabs and gather buffers of frame f and f+1
    are in flight together)."""
    cfg = scenes.CONFIGS["c3"]
    W, H = 1280, 720
    sc = cfg.scene()
    ctxs = [Tracer(0) for _ in range(n)]
    for c in ctxs:
        c.set_scene(sc)
    g = _group(ctxs, transport)
    try:
        info = [ctypes.c_int() for _ in range(4)]
        abi.check(abi.lib().rt_group_info(g, *[ctypes.byref(x) for x in info]), "rt_group_info")
        assert [x.value for x in info[:3]] == [n, n, 0]
        want_t = abi.RT_TRANSPORT_COPY if transport == abi.RT_TRANSPORT_AUTO and n > 1 else transport
        if transport == abi.RT_TRANSPORT_AUTO and n == 1:
            want_t = abi.RT_TRANSPORT_RCCL
        assert info[3].value == want_t
        cams = [cfg.camera(W, H), cfg.camera(W, H)]
        cams[1].eye = abi.vec3((30.0, 140.0, 260.0))
        tr.set_scene(sc)
        want = []
        for cam in cams:
            b = tr.render(cam, W, H, cfg.depth, rgba32f=True, rgba8=True)
            torch.cuda.synchronize()
            want.append((b["rgba32f"].clone(), b["rgba8"].clone()))
        s = torch.cuda.Stream()
        outs = [(torch.empty((H, W, 4), dtype=torch.float32, device="cuda"),
                 torch.empty((H, W, 4), dtype=torch.uint8, device="cuda")) for _ in range(6)]
        for f in range(6):
            _multi(g, cams[f % 2], W, H, cfg.depth, hb, outs[f][0], outs[f][1], s)
        s.synchronize()
        for f in range(6):
            assert torch.equal(outs[f][0], want[f % 2][0]), f"frame {f} RGBA32F differs"
            assert torch.equal(outs[f][1], want[f % 2][1]), f"frame {f} RGBA8 differs"
        # RGBA8 only (what the bench gathers)
        o8 = torch.empty((H, W, 4), dtype=torch.uint8, device="cuda")
        _multi(g, cams[0], W, H, cfg.depth, hb, None, o8, s)
        s.synchronize()
        assert torch.equal(o8, want[0][1])
    finally:
        abi.lib().rt_group_destroy(g)
        for c in ctxs:
            c.close()


def test_render_multi_c4_full_size_hash(tr):
    """c4 through rt_render_multi with 8 ranks: the assembled RGBA32F frame equals the float rounding of the
    single-GPU float64 frame, which hashes to the reference's own c3 frame."""
    cfg = scenes.CONFIGS["c3"]
    W, H = cfg.width, cfg.height
    sc = cfg.scene()
    ctxs = [Tracer(0) for _ in range(8)]
    for c in ctxs:
        c.set_scene(sc)
    g = _group(ctxs, abi.RT_TRANSPORT_AUTO)
    try:
        s = torch.cuda.Stream()
        o32 = torch.empty((H, W, 4), dtype=torch.float32, device="cuda")
        _multi(g, cfg.camera(), W, H, cfg.depth, 0, o32, None, s)
        s.synchronize()
        tr.set_scene(sc)
        b = tr.render(cfg.camera(), W, H, cfg.depth, rgba32f=False, rgb64f=True)
        torch.cuda.synchronize()
        rgb = b["rgb64f"].cpu().numpy()
        assert f"{po.fnv1a64(rgb):016x}" == golden.manifest()["frames"]["c3"]["fnv1a64"]
        assert np.array_equal(o32.cpu().numpy()[..., :3], rgb.astype(np.float32))
    finally:
        abi.lib().rt_group_destroy(g)
        for c in ctxs:
            c.close()


def test_group_errors_are_loud(tr):
    L = abi.lib()
    g = ctypes.c_void_p()
    arr = (ctypes.c_void_p * 2)(tr._ctx.value, tr._ctx.value)
    assert L.rt_group_create(arr, 2, abi.RT_TRANSPORT_AUTO, ctypes.byref(g)) == abi.RT_EINVAL   # same ctx twice
    other = Tracer(0)
    try:
        arr = (ctypes.c_void_p * 2)(tr._ctx.value, other._ctx.value)
        assert L.rt_group_create(arr, 2, abi.RT_TRANSPORT_RCCL, ctypes.byref(g)) == abi.RT_EINVAL  # one device
        assert "RCCL" in abi.last_error()
        g = _group([tr], abi.RT_TRANSPORT_COPY)
        cam = scenes.CONFIGS["c1"].camera(16, 16)
        assert L.rt_render_multi(g, ctypes.byref(cam), 16, 16, 1, 0, 0, None, None, None) == abi.RT_EINVAL
        assert L.rt_render_multi(g, ctypes.byref(cam), 16, 16, 1, 0, abi.RT_OUT_RGBA8, None, None, None) == abi.RT_EINVAL
        abi.lib().rt_group_destroy(g)
    finally:
        other.close()


def test_render_multi_rejects_local_contexts_with_different_scenes(tr):
    """A single-process group whose contexts hold different scenes — both achromatic, so the wire formats agree —
    fails with RT_EINVAL instead of assembling a frame from two scenes (one g_scene per frame, MSA:590); once
    both hold the same scene again the group renders the one-launch frame."""
    L = abi.lib()
    cfg = scenes.CONFIGS["c3"]
    W, H = 320, 180
    sc = cfg.scene()
    other = cfg.scene()
    other.spheres = other.spheres[:-1]                     # the same scene less its last sphere
    for s in (sc, other):
        flag = ctypes.c_int()
        abi.check(L.rt_scene_achromatic(ctypes.byref(s.to_abi()), ctypes.byref(flag)), "rt_scene_achromatic")
        assert flag.value == 1
    ctxs = [Tracer(0) for _ in range(2)]
    ctxs[0].set_scene(sc)
    ctxs[1].set_scene(other)
    g = _group(ctxs, abi.RT_TRANSPORT_COPY)
    try:
        cam = cfg.camera(W, H)
        o8 = torch.empty((H, W, 4), dtype=torch.uint8, device="cuda")
        s = torch.cuda.Stream()
        rc = L.rt_render_multi(g, ctypes.byref(cam), W, H, cfg.depth, 0, abi.RT_OUT_RGBA8, None, _ptr(o8),
                               ctypes.c_void_p(s.cuda_stream))
        assert rc == abi.RT_EINVAL
        assert "different scenes" in abi.last_error()
        ctxs[1].set_scene(sc)
        _multi(g, cam, W, H, cfg.depth, 0, None, o8, s)
        s.synchronize()
        tr.set_scene(sc)
        want = tr.render(cam, W, H, cfg.depth, rgba32f=False, rgba8=True)["rgba8"]
        torch.cuda.synchronize()
        assert torch.equal(o8, want)
    finally:
        L.rt_group_destroy(g)
        for c in ctxs:
            c.close()


def test_group_create_rank_one_process_per_gpu_path(tr):
    """The one-process-per-GPU constructor (rt_comm_unique_id + rt_group_create_rank, as bench.py uses under
    torch.distributed.run) with a one-rank communicator: same gather + assembly, equal to one launch."""
    L = abi.lib()
    cfg = scenes.CONFIGS["c2"]
    W, H = 640, 360
    uid = (ctypes.c_uint8 * abi.RT_COMM_ID_BYTES)()
    abi.check(L.rt_comm_unique_id(uid), "rt_comm_unique_id")
    t = Tracer(0)
    t.set_scene(cfg.scene())
    g = ctypes.c_void_p()
    abi.check(L.rt_group_create_rank(t._ctx, 1, 0, uid, ctypes.byref(g)), "rt_group_create_rank")
    try:
        info = [ctypes.c_int() for _ in range(4)]
        abi.check(L.rt_group_info(g, *[ctypes.byref(x) for x in info]), "rt_group_info")
        assert [x.value for x in info] == [1, 1, 0, abi.RT_TRANSPORT_RCCL]
        s = torch.cuda.Stream()
        o8 = torch.empty((H, W, 4), dtype=torch.uint8, device="cuda")
        cam = cfg.camera(W, H)
        for _ in range(3):
            _multi(g, cam, W, H, cfg.depth, 0, None, o8, s)
        abi.check(L.rt_group_synchronize(g), "rt_group_synchronize")
        s.synchronize()
        tr.set_scene(cfg.scene())
        want = tr.render(cam, W, H, cfg.depth, rgba32f=False, rgba8=True)["rgba8"]
        torch.cuda.synchronize()
        assert torch.equal(o8, want)
        assert L.rt_group_create_rank(t._ctx, 2, 2, uid, ctypes.byref(ctypes.c_void_p())) == abi.RT_EINVAL
    finally:
        L.rt_group_destroy(g)
        t.close()


def _read_ppm(path):
    data = open(path, "rb").read()
    parts = data.split(b"\n", 1)
    hdr = parts[0].split()
    assert hdr[0] == b"P6" and hdr[3] == b"255"
    W, H = int(hdr[1]), int(hdr[2])
    return np.frombuffer(parts[1], np.uint8).reshape(H, W, 3)


@pytest.mark.parametrize("gpus", [1, 4, 8])
def test_cli_gpus_ppm_equals_single(tmp_path, gpus):
    """`rt_render --config c4 --gpus N` (rt_group + rt_render_multi from C++) writes the same PPM as the
    one-launch `rt_render --config c3`."""
    exe = os.path.join(LIBDIR, "rt_render")
    one, multi = tmp_path / "c3.ppm", tmp_path / "c4.ppm"
    r = subprocess.run([exe, "--config", "c3", "--out", str(one)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    r = subprocess.run([exe, "--config", "c4", "--gpus", str(gpus), "--repeat", "3", "--out", str(multi)],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert f"over {gpus} ranks" in r.stdout
    assert ("RCCL" if gpus == 1 else "device-copy") in r.stdout
    assert np.array_equal(_read_ppm(one), _read_ppm(multi))


def test_dropin_binding_demo_board(tmp_path):
    """INTEGRATION.md's loadScene/draw()/writePpmScreenshot binding (csrc/rt_dropin.cpp, built against
    rt_api.h and the real GL headers) on initScene's demo board: light b6, tetrahedron b4, sphere d7,
    cube a7, at the app's 500x500 window, unit pitch, MAX_DEPTH 5 — equal to the oracle's frame."""
    exe = os.path.join(LIBDIR, "rt_dropin")
    out = tmp_path / "dropin.ppm"
    r = subprocess.run([exe, "--frames", "5", "--out", str(out), "b6:a", "b4:b", "d7:d", "a7:c"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "5 frame(s)" in r.stdout
    sc = scenes.load_scene([("b6", scenes.LIGHT), ("b4", scenes.TETRAHEDRON), ("d7", scenes.SPHERE),
                            ("a7", scenes.CUBE)])
    want, _ = po.render(sc.to_abi(), scenes.make_camera(500, 500, 1.0), 500, 500, 5)
    q = np.floor(np.clip(want, 0.0, 1.0) * 255.0 + 0.5).astype(np.uint8)[::-1]
    assert np.array_equal(_read_ppm(out), q)


@pytest.mark.parametrize("opts", [["--format", "gray"], ["--pipelined"], ["--pageable", "--format", "rgba"],
                                  ["--pipelined", "--pageable", "--format", "rgb"]])
def test_dropin_binding_formats_and_pipelining(tmp_path, opts):
    """The binding's frame formats (GRAY8 for the achromatic board: light, tetrahedron, spheres — no red cube),
    pinned / pageable buffers and the pipelined draw() (the PPM is the last queued frame): the PPM equals the
    oracle's frame, quantised, whatever crossed PCIe."""
    exe = os.path.join(LIBDIR, "rt_dropin")
    out = tmp_path / "dropin.ppm"
    entries = ["b6:a", "b4:b", "d7:d", "f3:d"]
    r = subprocess.run([exe, "--frames", "4", "--width", "320", "--height", "240", "--pitch", "1.5", "--out", str(out)]
                       + opts + entries, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    if opts == ["--pipelined"]:
        assert "GRAY8" in r.stdout and "pipelined" in r.stdout        # auto: achromatic board -> GRAY8
    sc = scenes.load_scene([("b6", scenes.LIGHT), ("b4", scenes.TETRAHEDRON), ("d7", scenes.SPHERE),
                            ("f3", scenes.SPHERE)])
    want, _ = po.render(sc.to_abi(), scenes.make_camera(320, 240, 1.5), 320, 240, 5)
    q = np.floor(np.clip(want, 0.0, 1.0) * 255.0 + 0.5).astype(np.uint8)[::-1]
    assert np.array_equal(_read_ppm(out), q)


def _devices():
    return torch.cuda.device_count() if torch.cuda.is_available() else 0


@pytest.mark.skipif(_devices() < 2, reason="needs >= 2 GPUs: the RCCL send/recv gather over distinct devices "
                                           "(ncclCommInitAll) cannot run on a one-GPU box")
@pytest.mark.parametrize("outputs", ["rgba8", "both"])
def test_render_multi_rccl_distinct_devices(outputs):
    """c4 over RCCL for real: one context per device (rt_group_create -> ncclCommInitAll), N = 2 ..
    device_count ranks, 3840x2160 c3 frames with alternating eyes (double buffers in flight); rank 0's images
    equal a one-launch render byte for byte, and the float64 one-launch frame hashes to the reference's c3."""
    cfg = scenes.CONFIGS["c3"]
    W, H = cfg.width, cfg.height
    sc = cfg.scene()
    one = Tracer(0)
    one.set_scene(sc)
    cams = [cfg.camera(), cfg.camera()]
    cams[1].eye = abi.vec3((30.0, 140.0, 260.0))
    want = []
    for cam in cams:
        b = one.render(cam, W, H, cfg.depth, rgba32f=True, rgba8=True, rgb64f=cam is cams[0])
        torch.cuda.synchronize()
        want.append(b)
    assert f"{po.fnv1a64(want[0]['rgb64f'].cpu().numpy()):016x}" == golden.manifest()["frames"]["c3"]["fnv1a64"]
    for n in sorted({2, min(4, _devices()), _devices()}):
        ctxs = [Tracer(d) for d in range(n)]
        for c in ctxs:
            c.set_scene(sc)
        g = _group(ctxs, abi.RT_TRANSPORT_RCCL)
        try:
            info = [ctypes.c_int() for _ in range(4)]
            abi.check(abi.lib().rt_group_info(g, *[ctypes.byref(x) for x in info]), "rt_group_info")
            assert [x.value for x in info] == [n, n, 0, abi.RT_TRANSPORT_RCCL]
            abi.check(abi.lib().rt_group_timing(g, 1), "rt_group_timing")
            with torch.cuda.device(0):
                s = torch.cuda.Stream()
                outs = [(torch.empty((H, W, 4), dtype=torch.float32, device="cuda:0") if outputs == "both" else None,
                         torch.empty((H, W, 4), dtype=torch.uint8, device="cuda:0")) for _ in range(6)]
                for f in range(6):
                    _multi(g, cams[f % 2], W, H, cfg.depth, 0, outs[f][0], outs[f][1], s)
                s.synchronize()
            abi.check(abi.lib().rt_group_synchronize(g), "rt_group_synchronize")
            for f in range(6):
                assert torch.equal(outs[f][1], want[f % 2]["rgba8"]), (n, f)
                if outputs == "both":
                    assert torch.equal(outs[f][0], want[f % 2]["rgba32f"]), (n, f)
            st = abi.rt_group_stats()
            abi.check(abi.lib().rt_group_get_stats(g, ctypes.byref(st)), "rt_group_get_stats")
            assert st.wire_byte == abi.RT_PIXEL_GRAY8 and st.ranks_timed == n and st.gather_ms > 0
            print(f"n={n}: render {st.render_ms:.3f} ms, gather {st.gather_ms:.3f} ms, assemble "
                  f"{st.assemble_ms:.3f} ms, frame {st.frame_ms:.3f} ms, payload {st.payload_bytes} B")
        finally:
            abi.lib().rt_group_destroy(g)
            for c in ctxs:
                c.close()
    one.close()


def test_dropin_rejects_cylinder(tmp_path):
    exe = os.path.join(LIBDIR, "rt_dropin")
    r = subprocess.run([exe, "--out", str(tmp_path / "x.ppm"), "b6:a", "c3:e"], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 1 and "cylinder" in r.stderr.lower()


def test_render_host_repeated_calls_reuse_state(tr):
    """rt_render called every frame (draw()): an unchanged scene is not re-uploaded, the device buffers are
    reused, and every call's image and ray statistics (summed on the device) are the oracle's."""
    cfg = scenes.CONFIGS["c2"]
    sa = cfg.scene().to_abi()
    W, H = 480, 270
    cam = cfg.camera(W, H)
    want, want_rc = po.render(sa, cam, W, H, cfg.depth)
    total = int((want_rc & 0xFFFF).sum()) + int((want_rc >> 16).sum())
    for k in range(4):
        rgb, st = tr.render_host(sa, cam, W, H, cfg.depth)
        assert np.array_equal(rgb, want), f"call {k}"
        assert st.primary_rays == W * H
        assert st.primary_rays + st.reflect_rays + st.shadow_rays == total
    # a different scene through the same context, then the first one again
    sb = scenes.CONFIGS["c1"].scene().to_abi()
    rgb, _ = tr.render_host(sb, cam, W, H, 0)
    assert np.array_equal(rgb, po.render(sb, cam, W, H, 0)[0])
    rgb, _ = tr.render_host(sa, cam, W, H, cfg.depth)
    assert np.array_equal(rgb, want)


def test_set_scene_waits_for_renders_on_other_streams(tr):
    """rt_set_scene right after renders queued on a non-blocking stream: the queued renders still see the
    old scene (the upload waits for them), later renders the new one."""
    W, H = 960, 540
    a, b = scenes.CONFIGS["c5"], scenes.CONFIGS["c1"]
    cam = a.camera(W, H)
    s = torch.cuda.Stream()
    tr.set_scene(a.scene())
    bufs = [tr.alloc(W, H, rgba32f=False, rgb64f=True) for _ in range(3)]
    for k in range(3):
        tr.render_into(cam, W, H, 2, bufs[k], stream=s)
    tr.set_scene(b.scene())
    s.synchronize()
    want_a, _ = po.render(a.scene().to_abi(), cam, W, H, 2)
    for k in range(3):
        assert np.array_equal(bufs[k]["rgb64f"].cpu().numpy(), want_a), f"render {k} saw the new scene"
    nb = tr.render(cam, W, H, 2, rgba32f=False, rgb64f=True)
    torch.cuda.synchronize()
    assert np.array_equal(nb["rgb64f"].cpu().numpy(), po.render(b.scene().to_abi(), cam, W, H, 2)[0])


def test_graph_replay_after_other_views(tr):
    """A captured render replays bit-exact after the context rendered other eyes and sizes (its per-eye data
    and tile order are carried in the graph), and renders after the capture stay exact too."""
    cfg = scenes.CONFIGS["c5"]
    W, H = 320, 200
    cam = cfg.camera(W, H)
    tr.set_scene(cfg.scene())
    bufs = tr.alloc(W, H, rgba32f=False, rgb64f=True)
    s = torch.cuda.Stream()
    for _ in range(3):                                  # the view's order is calibrated before the capture
        tr.render_into(cam, W, H, 2, bufs, stream=s)
    s.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        tr.render_into(cam, W, H, 2, bufs, stream=s)
    want, _ = po.render(cfg.scene().to_abi(), cam, W, H, 2)
    other = cfg.camera(W + 40, H + 24)
    other.eye = abi.vec3((-80.0, 60.0, 150.0))
    want_o, _ = po.render(cfg.scene().to_abi(), other, W + 40, H + 24, 2)
    for k in range(3):
        for _ in range(3):                              # another eye and size, long enough to be calibrated
            ob = tr.render(other, W + 40, H + 24, 2, rgba32f=False, rgb64f=True)
        torch.cuda.synchronize()
        assert np.array_equal(ob["rgb64f"].cpu().numpy(), want_o)
        bufs["rgb64f"].zero_()
        g.replay()
        torch.cuda.synchronize()
        assert np.array_equal(bufs["rgb64f"].cpu().numpy(), want), f"replay {k}"


@pytest.mark.parametrize("policy", ["identity", "stale_order"])
def test_moving_camera_reuses_order_exactly(tr, monkeypatch, policy):
    """A camera that moves every frame, with a calibrated view of the same frame shape before it: by default (r06)
    each new view renders in identity order (and a view rendered twice is calibrated); with RT_MOVING_ORDER=1 the
    renders reuse the last calibrated tile-row order and re-time it every 8th frame (RT_RECALIBRATE, the r03-r05
    policy).  Every frame stays the oracle's, and so does a size change in the middle (a new shape: identity order,
    then calibration)."""
    if policy == "stale_order":
        monkeypatch.setenv("RT_MOVING_ORDER", "1")
        monkeypatch.setenv("RT_RECALIBRATE", "8")
    t = Tracer(0)
    cfg = scenes.CONFIGS["c2"]
    sc = cfg.scene()
    t.set_scene(sc)
    sa = sc.to_abi()
    try:
        for (W, H) in ((320, 180), (256, 200)):
            for _ in range(3):                          # the static view first: calibrated
                t.render(cfg.camera(W, H), W, H, cfg.depth, rgba32f=False, rgb64f=True)
            for v in range(20):
                cam = cfg.camera(W, H)
                ang = 2.0 * np.pi * v / 20
                cam.eye = abi.vec3((60.0 * np.sin(ang), 100.0 + 10.0 * np.cos(ang), 200.0))
                b = t.render(cam, W, H, cfg.depth, rgba32f=False, rgb64f=True, raycount=True)
                torch.cuda.synchronize()
                want, want_rc = po.render(sa, cam, W, H, cfg.depth)
                assert np.array_equal(b["rgb64f"].cpu().numpy(), want), (W, v)
                assert np.array_equal(b["raycount"].cpu().numpy().view(np.uint32), want_rc), (W, v)
    finally:
        t.close()
