"""GPU tests of the per-view primary cone-mask cache (rt_kernel.hip render_dev_impl, rt_disp_kernel):
the calibration render of a static view records each 8x8 tile's primary-ray sphere mask, later renders of
exactly that view read it (one scalar load) instead of recomputing it, and renders of any other camera
compute their own.  The masks only skip spheres a tile's rays provably miss, so every frame must stay
bit-exact with the reference (MySdlApplication.cpp:1184-1249 via the golden manifest) whichever path made
its mask — first render, calibration, cached, other camera, back to the cached view, across streams."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

from oracle import pyoracle as po  # noqa: E402
from ray_tracer_fragment_shader_amd import abi, scenes  # noqa: E402
from ray_tracer_fragment_shader_amd.tracer import Tracer  # noqa: E402

from . import golden  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def tr():
    if not torch.cuda.is_available():
        pytest.fail("gpu tests need a HIP device")
    t = Tracer(0)
    yield t
    t.close()


def _hash(b):
    return f"{po.fnv1a64(b['rgb64f'].cpu().numpy()):016x}"


def _moved(cfg, ang):
    cam = cfg.camera()
    cam.eye = abi.vec3((60.0 * np.sin(ang), 100.0 + 10.0 * np.cos(ang), 200.0))
    return cam


@pytest.mark.parametrize("name", ["c2", "c3", "c5"])
def test_static_view_frames_hash_to_the_reference(tr, name):
    """Renders 1 (identity order, masks computed), 2 (calibration: masks recorded) and 3-5 (masks read from the
    cache, longest-first order) of one view: every frame is the reference's (manifest hash)."""
    cfg = scenes.CONFIGS[name]
    tr.set_scene(cfg.scene())
    want = golden.manifest()["frames"][name]["fnv1a64"]
    for k in range(5):
        b = tr.render(cfg.camera(), cfg.width, cfg.height, cfg.depth, rgba32f=False, rgb64f=True)
        torch.cuda.synchronize()
        assert _hash(b) == want, f"render {k}"


@pytest.mark.parametrize("name", ["c2", "c5"])
def test_tile_order_policy_frames_hash_to_the_reference(monkeypatch, name):
    """The per-tile longest-first dispatch order (RT_ORDER_POLICY=1: tile costs sorted by hipCUB into the dispatch
    records) instead of the tile-row order: the first, calibration and cached renders all hash to the reference."""
    monkeypatch.setenv("RT_ORDER_POLICY", "1")
    cfg = scenes.CONFIGS[name]
    t = Tracer(0)
    try:
        t.set_scene(cfg.scene())
        want = golden.manifest()["frames"][name]["fnv1a64"]
        for k in range(4):
            b = t.render(cfg.camera(), cfg.width, cfg.height, cfg.depth, rgba32f=False, rgb64f=True)
            torch.cuda.synchronize()
            assert _hash(b) == want, f"render {k}"
    finally:
        t.close()


def test_other_cameras_and_back(tr):
    """A cached view, then cameras of the same frame shape (their own masks; identity order by default, the
    calibrated order reused and re-timed every 8th render with RT_MOVING_ORDER=1), then the cached view again: each
    frame equals a fresh context's first render of that camera, and the cached view still hashes to the reference."""
    cfg = scenes.CONFIGS["c2"]
    W, H = cfg.width, cfg.height
    sc = cfg.scene()
    tr.set_scene(sc)
    want = golden.manifest()["frames"]["c2"]["fnv1a64"]
    for _ in range(3):
        b = tr.render(cfg.camera(), W, H, cfg.depth, rgba32f=False, rgb64f=True)
    views = [_moved(cfg, 2.0 * np.pi * v / 12) for v in range(12)]
    got = []
    for v in views:
        b = tr.render(v, W, H, cfg.depth, rgba32f=False, rgb64f=True)
        got.append(b["rgb64f"].clone())
    b = tr.render(cfg.camera(), W, H, cfg.depth, rgba32f=False, rgb64f=True)
    torch.cuda.synchronize()
    assert _hash(b) == want
    fresh = Tracer(0)
    try:
        fresh.set_scene(sc)
        for v, g in zip(views, got):
            ref = fresh.render(v, W, H, cfg.depth, rgba32f=False, rgb64f=True)["rgb64f"]
            torch.cuda.synchronize()
            assert torch.equal(g, ref)
    finally:
        fresh.close()


def test_view_change_with_renders_in_flight_on_other_streams(tr):
    """Cached renders of view A queued on one stream, then view B rendered twice on another stream (its
    calibration rewrites the cache while A's renders may still be running: the context drains the device
    first), then A again: every A frame hashes to the reference, B equals a fresh context's render."""
    cfg = scenes.CONFIGS["c3"]
    W, H = cfg.width, cfg.height
    sc = cfg.scene()
    tr.set_scene(sc)
    want = golden.manifest()["frames"]["c3"]["fnv1a64"]
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    for _ in range(3):
        tr.render(cfg.camera(), W, H, cfg.depth, rgba32f=False, rgb64f=True, stream=s1)
    torch.cuda.synchronize()
    bufs = [tr.alloc(W, H, rgba32f=False, rgb64f=True) for _ in range(4)]
    for b in bufs[:3]:
        tr.render_into(cfg.camera(), W, H, cfg.depth, b, stream=s1)
    vb = _moved(cfg, 1.0)
    tr.render(vb, W, H, cfg.depth, rgba32f=False, rgb64f=True, stream=s2)
    b_frame = tr.render(vb, W, H, cfg.depth, rgba32f=False, rgb64f=True, stream=s2)
    tr.render_into(cfg.camera(), W, H, cfg.depth, bufs[3], stream=s1)
    torch.cuda.synchronize()
    for k, b in enumerate(bufs):
        assert _hash(b) == want, f"A frame {k}"
    fresh = Tracer(0)
    try:
        fresh.set_scene(sc)
        ref = fresh.render(vb, W, H, cfg.depth, rgba32f=False, rgb64f=True)["rgb64f"]
        torch.cuda.synchronize()
        assert torch.equal(b_frame["rgb64f"], ref)
    finally:
        fresh.close()


@pytest.mark.parametrize("name", ["c2", "c3"])
def test_calibrate_on_one_stream_read_on_another(name):
    """The calibration render (and the order / mask-permute kernels after it) queued on s1, then at once — no
    synchronisation — cached renders of the same view on s2 and s3: they must wait for the calibration's buffers
    on the GPU (the context's calibration event), and every frame hashes to the reference.  Then a view change
    calibrated on s2 while s3's cached renders may still be reading: A frames stay exact, B equals a fresh render."""
    cfg = scenes.CONFIGS[name]
    W, H = cfg.width, cfg.height
    sc = cfg.scene()
    want = golden.manifest()["frames"][name]["fnv1a64"]
    t = Tracer(0)
    try:
        t.set_scene(sc)
        s1, s2, s3 = torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()
        bufs = [t.alloc(W, H, rgba32f=False, rgb64f=True) for _ in range(6)]
        t.render_into(cfg.camera(), W, H, cfg.depth, bufs[0], stream=s1)      # first render: identity order
        torch.cuda.synchronize()
        t.render_into(cfg.camera(), W, H, cfg.depth, bufs[1], stream=s1)      # calibration (not waited for)
        t.render_into(cfg.camera(), W, H, cfg.depth, bufs[2], stream=s2)      # cached, another stream
        t.render_into(cfg.camera(), W, H, cfg.depth, bufs[3], stream=s3)
        t.render_into(cfg.camera(), W, H, cfg.depth, bufs[4], stream=s3)
        vb = _moved(cfg, 0.7)
        b0 = t.render(vb, W, H, cfg.depth, rgba32f=False, rgb64f=True, stream=s2)
        b1 = t.render(vb, W, H, cfg.depth, rgba32f=False, rgb64f=True, stream=s2)    # calibrates B on s2
        t.render_into(cfg.camera(), W, H, cfg.depth, bufs[5], stream=s1)
        torch.cuda.synchronize()
        for k, b in enumerate(bufs):
            assert _hash(b) == want, f"A frame {k}"
        fresh = Tracer(0)
        try:
            fresh.set_scene(sc)
            ref = fresh.render(vb, W, H, cfg.depth, rgba32f=False, rgb64f=True)["rgb64f"]
            torch.cuda.synchronize()
            assert torch.equal(b0["rgb64f"], ref) and torch.equal(b1["rgb64f"], ref)
        finally:
            fresh.close()
    finally:
        t.close()


def _random_cull_scene(rng, n_spheres, n_lights):
    sq = [chr(ord("a") + int(rng.integers(0, 8))) + chr(ord("1") + int(rng.integers(0, 8))) for _ in range(n_spheres)]
    sph = [scenes.SphereSpec(s, float(rng.uniform(2, 30)), float(rng.uniform(-40, 90))) for s in sq]
    lts = [scenes.LightSpec(chr(ord("a") + int(rng.integers(0, 8))) + chr(ord("1") + int(rng.integers(0, 8))),
                            scenes.WHITE if k % 2 == 0 else tuple(float(x) for x in rng.uniform(0, 1, 3)))
           for k in range(n_lights)]
    return scenes.Scene(spheres=sph, lights=lts)


@pytest.mark.parametrize("seed,n_spheres,n_lights,depth", [(0, 20, 1, 2), (1, 40, 2, 3), (2, 64, 3, 5),
                                                           (3, 33, 2, 7), (4, 48, 4, 5), (5, 8, 1, 1), (6, 12, 2, 2),
                                                           (7, 9, 3, 4), (8, 6, 2, 3), (9, 3, 1, 2)])
def test_level_mask_cache_random_culling_scenes(seed, n_spheres, n_lights, depth):
    """Per-tile level masks (rt_device.hpp LevelMasks): the calibration of a static view stores every level's ray and
    shadow masks — the culling kernels (>= 16 spheres) in the calibration render itself, the fast kernels' scenes
    (8-15 padded spheres) through a culling launch of its own — and later renders of that view read them (the fast
    kernels skip the filter batches they rule out).  Random scenes, 1-4 lights, depth 1-7, including slot counts past
    the cache's limit (seed 3: 7 + 8 x 2 = 23 slots, cached; seed 4: 5 + 6 x 4 = 29, computed) and a scene below the
    primary cone's 8 spheres (seed 9: no masks): the first, calibration and cached renders equal the oracle bit for
    bit."""
    rng = np.random.default_rng(seed)
    sc = _random_cull_scene(rng, n_spheres, n_lights)
    W, H = 160, 120
    cam = scenes.make_camera(W, H, float(rng.uniform(1.0, 3.0)))
    want, want_rc = po.render(sc.to_abi(), cam, W, H, depth)
    t = Tracer(0)
    try:
        t.set_scene(sc)
        for k in range(5):
            b = t.render(cam, W, H, depth, rgba32f=False, rgb64f=True, raycount=True)
            torch.cuda.synchronize()
            assert np.array_equal(b["rgb64f"].cpu().numpy(), want, equal_nan=True), f"render {k}"
            assert np.array_equal(b["raycount"].cpu().numpy().view(np.uint32), want_rc), f"render {k}"
        # the bench's output set (RGBA32F + RGBA8): its own calibration and cached renders equal the first
        first = t.render(cam, W, H, depth, rgba32f=True, rgba8=True)
        torch.cuda.synchronize()
        ref = (first["rgba32f"].clone(), first["rgba8"].clone())
        for k in range(3):
            b = t.render(cam, W, H, depth, rgba32f=True, rgba8=True)
            torch.cuda.synchronize()
            assert torch.equal(b["rgba32f"], ref[0]) and torch.equal(b["rgba8"], ref[1]), f"rgba render {k}"
    finally:
        t.close()


def test_level_mask_cache_off_and_view_changes(monkeypatch):
    """c5 (64 spheres, 2 lights, depth 3) at 640x360: a context without the level-mask cache (RT_LEVEL_MASKS=0) and one
    with it render the same frames; then the cached context renders another camera (masks computed in the kernel, the
    calibrated order reused) and the cached view again — every frame equals the uncached context's."""
    cfg = scenes.CONFIGS["c5"]
    W, H = 640, 360
    monkeypatch.setenv("RT_LEVEL_MASKS", "0")
    off = Tracer(0)
    monkeypatch.delenv("RT_LEVEL_MASKS")
    on = Tracer(0)
    try:
        for t in (off, on):
            t.set_scene(cfg.scene())
        cams = [cfg.camera(W, H), cfg.camera(W, H)]
        cams[1].eye = abi.vec3((60.0 * np.sin(0.7), 100.0 + 10.0 * np.cos(0.7), 200.0))
        seq = [0, 0, 0, 0, 1, 1, 0, 0]
        for k, ci in enumerate(seq):
            a = off.render(cams[ci], W, H, cfg.depth, rgba32f=True, rgba8=True)
            b = on.render(cams[ci], W, H, cfg.depth, rgba32f=True, rgba8=True)
            torch.cuda.synchronize()
            assert torch.equal(a["rgba32f"], b["rgba32f"]) and torch.equal(a["rgba8"], b["rgba8"]), f"frame {k}"
    finally:
        off.close()
        on.close()
