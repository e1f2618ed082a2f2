"""The sun exit tables on the GPU (DESIGN.md §3 "Sun exit tables"): the copy a
frame reads (vx_prepare_sun) is the one the oracle's restatement of the rule
picks; frames are bit-identical with the tables, with the orthant copies only
and with none, over suns that need new cone copies (the scene keeps two, so
the third evicts one) and frames in flight on two streams right after a sun
change; the work counters equal the oracle's with the same tables."""
import math

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _gpu():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:  # pragma: no cover
        return False


@pytest.fixture(scope="module", autouse=True)
def _need_gpu(built):
    if not _gpu():
        pytest.skip("no GPU visible")


@pytest.fixture(scope="module")
def scene(noise):
    import voxmap_amd as vx
    from voxmap_amd import scenes
    dims = (128, 64, 24)
    field = vx.field_build(scenes.small_proc(31, dims=dims, n_boxes=20, n_glass=5))
    sc = vx.Scene(map_bytes=field.tobytes(), map_format=vx.FORMAT_BIN, noise_bytes=noise.tobytes(),
                  noise_format=vx.FORMAT_BIN, dims=dims, device=0)
    yield sc, field
    sc.close()


def _sun(el_deg, az_deg):
    el, az = math.radians(el_deg), math.radians(az_deg)
    return (math.cos(el) * math.cos(az), math.cos(el) * math.sin(az), math.sin(el))


# (elevation, azimuth): windows (kx, ky) = (2, 1), (1, 2), (1, 1), (4, 4) in
# different octants, a low sun (orthant copies) and a sun below the horizon
SUNS = [(33, 30), (40, 120), (60, 210), (20, 300), (10, 45), (-20, 80)]


@pytest.mark.parametrize("el,az", SUNS)
def test_prepare_sun_matches_the_oracle_rule(scene, el, az):
    import oracle
    import voxmap_amd as vx
    sc, _ = scene
    sun = _sun(el, az)
    fr = vx.make_frame((64.0, 32.0, 30.0), (1.0, 0.0, 0.6), 96, 64, sun=sun)
    info = sc.prepare_sun(fr)
    cone, octs, kx, ky = oracle.exit_plan([fr.params.sun_dir[:]])
    if el < 0:
        assert info["kind"] == 1 or info["kind"] == 0    # below the horizon: shadeFactor is 0 anyway
    elif cone:
        assert (info["kind"], info["octant"], info["kx"], info["ky"]) == (2, octs[0], kx, ky)
    else:
        assert (info["kind"], info["octant"]) == (1, octs[0])
    fr.params.flags |= vx.FLAG_NO_EXIT
    assert sc.prepare_sun(fr)["kind"] == 0


def test_frames_identical_across_sun_changes_and_table_modes(scene, noise):
    """Cycle through suns needing four different copies (two cache slots: every
    new one evicts), render each with cone, orthant and no tables: identical
    RGBA32F frames, and counters equal to the oracle's with the same tables."""
    import oracle
    import voxmap_amd as vx
    sc, field = scene
    o = oracle.Oracle(sc.read_field(), noise, exit=True)
    for rep in range(2):
        for el, az in SUNS[:4] + SUNS[:2]:
            sun = _sun(el, az)
            fr = vx.make_frame((40.0, 20.0, 26.0), (1.1, 0.0, 0.5 + 0.3 * rep), 128, 72, sun=sun,
                               flags=vx.FLAG_FULL_QUALITY)
            img, st = sc.render(fr, stats=True)
            ref, ost = o.render(fr.params, 128, 72)
            assert np.array_equal(img.view(np.uint32), ref.view(np.uint32)), (el, az)
            assert st.as_dict()["shadow_fetches"] == ost.as_dict()["shadow_fetches"]
            for fl in (vx.FLAG_NO_CONE, vx.FLAG_NO_EXIT):
                f2 = vx.make_frame((40.0, 20.0, 26.0), (1.1, 0.0, 0.5 + 0.3 * rep), 128, 72, sun=sun,
                                   flags=vx.FLAG_FULL_QUALITY | fl)
                img2 = sc.render(f2)
                if isinstance(img2, tuple):
                    img2 = img2[0]
                assert np.array_equal(img2.view(np.uint32), img.view(np.uint32)), (el, az, fl)


def test_two_streams_right_after_a_sun_change(scene):
    """A new sun's cone copy is built on the first frame's stream; a frame
    launched at once on a second stream must wait for it (hipStreamWaitEvent):
    both RGBA8 frames equal the single-stream frame, for several sun changes."""
    import torch

    import voxmap_amd as vx
    sc, _ = scene
    W, H = 256, 160
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    a = torch.empty(W * H * 4, dtype=torch.uint8, device="cuda")
    b = torch.empty_like(a)
    for el, az in [(25, 15), (35, 140), (50, 250), (28, 320), (25, 15)]:
        fr = vx.make_frame((64.0, 32.0, 34.0), (1.0, 0.0, -0.4), W, H, sun=_sun(el, az),
                           flags=vx.FLAG_FULL_QUALITY)
        sc.render_device(fr, a.data_ptr(), pixel_format=vx.PIXEL_RGBA8, stream=s1.cuda_stream)
        sc.render_device(fr, b.data_ptr(), pixel_format=vx.PIXEL_RGBA8, stream=s2.cuda_stream)
        torch.cuda.synchronize()
        ref = sc.render(fr, pixel_format=vx.PIXEL_RGBA8)
        if isinstance(ref, tuple):
            ref = ref[0]
        ref = np.ascontiguousarray(ref).view(np.uint8).ravel()
        assert np.array_equal(a.cpu().numpy(), ref), (el, az)
        assert np.array_equal(b.cpu().numpy(), ref), (el, az)


def test_two_threads_cycle_three_suns(scene):
    """two host threads render one scene on their own streams while
    cycling through three suns with different cone windows (two cache slots, so
    slots are recycled while the other thread's frames may still read them).
    A slot is pinned from its lookup until the render that reads it is enqueued,
    and a recycle waits for the device, so every render that read the slot has
    finished (vx_api.cpp cone_copy; no caller stream handle is kept).
    Every frame equals the same frame rendered alone."""
    import threading

    import torch

    import voxmap_amd as vx
    sc, _ = scene
    W, H = 192, 120
    suns = [(33, 30), (40, 120), (60, 210)]
    frames = {k: vx.make_frame((64.0, 32.0, 34.0), (1.0, 0.0, -0.4), W, H, sun=_sun(*k),
                               flags=vx.FLAG_FULL_QUALITY) for k in suns}
    refs = {}
    for k, fr in frames.items():
        r = sc.render(fr, pixel_format=vx.PIXEL_RGBA8)
        refs[k] = np.ascontiguousarray(r[0] if isinstance(r, tuple) else r).view(np.uint8).ravel()
    errors = []

    def worker(tid):
        try:
            st = torch.cuda.Stream()
            bufs = [torch.empty(W * H * 4, dtype=torch.uint8, device="cuda") for _ in range(3)]
            for rep in range(12):
                order = suns if tid == 0 else suns[::-1]
                for j, k in enumerate(order):
                    sc.render_device(frames[k], bufs[j].data_ptr(), pixel_format=vx.PIXEL_RGBA8,
                                     stream=st.cuda_stream)
                st.synchronize()
                for j, k in enumerate(order):
                    if not np.array_equal(bufs[j].cpu().numpy(), refs[k]):
                        errors.append((tid, rep, k))
        except Exception as e:  # pragma: no cover - reported below
            errors.append((tid, repr(e)))

    ts = [threading.Thread(target=worker, args=(i,)) for i in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errors, errors[:5]


def test_two_threads_per_thread_stream_cycle_three_suns(scene):
    """hipStreamPerThread is one handle that names a different
    stream on each host thread.  Two threads pass it while cycling three cone
    windows through the two slots: a slot is recycled only after a device-wide
    wait, and a cache hit waits for the build until the host has seen it
    complete.  Every frame equals the frame rendered alone."""
    import threading

    import torch

    import voxmap_amd as vx
    sc, _ = scene
    W, H = 192, 120
    per_thread = 2                                   # hipStreamPerThread (hip_runtime_api.h)
    suns = [(31, 40), (44, 130), (57, 220)]
    frames = {k: vx.make_frame((64.0, 32.0, 34.0), (1.0, 0.0, -0.4), W, H, sun=_sun(*k),
                               flags=vx.FLAG_FULL_QUALITY) for k in suns}
    refs = {}
    for k, fr in frames.items():
        r = sc.render(fr, pixel_format=vx.PIXEL_RGBA8)
        refs[k] = np.ascontiguousarray(r[0] if isinstance(r, tuple) else r).view(np.uint8).ravel()
    errors = []

    def worker(tid):
        try:
            bufs = [torch.empty(W * H * 4, dtype=torch.uint8, device="cuda") for _ in range(3)]
            for rep in range(10):
                order = suns if tid == 0 else suns[::-1]
                for j, k in enumerate(order):
                    sc.render_device(frames[k], bufs[j].data_ptr(), pixel_format=vx.PIXEL_RGBA8, stream=per_thread)
                torch.cuda.synchronize()
                for j, k in enumerate(order):
                    if not np.array_equal(bufs[j].cpu().numpy(), refs[k]):
                        errors.append((tid, rep, k))
        except Exception as e:  # pragma: no cover - reported below
            errors.append((tid, repr(e)))

    ts = [threading.Thread(target=worker, args=(i,)) for i in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errors, errors[:5]


@pytest.mark.parametrize("flags", [48], ids=["full"])
def test_c3_full_size_no_exit_equals_exit_tables(noise, flags):
    """VERDICT r03 housekeeping: the bench's C3 K1 frame (3840x2160, full
    quality) marched without the exit tables (VX_FLAG_NO_EXIT: every step of
    render.frag:92-136) equals the exit-table frame bit for bit, and its shadow
    fetch count is the oracle's literal march's."""
    import oracle
    import voxmap_amd as vx
    from voxmap_amd import presets
    field = vx.field_build(presets.scene_grid("s_proc"))
    with vx.Scene(map_bytes=field.tobytes(), map_format=vx.FORMAT_BIN, noise_bytes=noise.tobytes(),
                  noise_format=vx.FORMAT_BIN, dims=(1024, 256, 32), device=0) as sc:
        fr = presets.camera_frame("K1", 3840, 2160, flags=flags)
        a, sa = sc.render(fr, stats=True)
        fn = presets.camera_frame("K1", 3840, 2160, flags=flags | vx.FLAG_NO_EXIT)
        b, sb = sc.render(fn, stats=True)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
    assert sb.shadow_fetches > 3 * sa.shadow_fetches
    _, ost = oracle.Oracle(field, noise).render(fn.params, 3840, 2160, row0=0, row_step=1, threads=16)
    assert sb.shadow_fetches == ost.shadow_fetches and sb.primary_fetches == ost.primary_fetches


# ---- full-size evidence that the exit tables change no pixel ----
def _literal_subset(sc, fr, W, H, O, every=16):
    """The frame marched WITHOUT exit tables (VX_FLAG_NO_EXIT, every step of
    render.frag:92-136) on a band subset (8-row bands 0, every, 2*every, ...:
    rows j + 8*every*k, j < 8) against the oracle's literal march
    (Oracle(exit=False)) on the same rows: every fp32 word and every work
    counter.  Returns the device's subset rows."""
    import torch

    import voxmap_amd as vx
    assert fr.params.flags & vx.FLAG_NO_EXIT
    ids = list(range(0, -(-H // 8), every))
    out = torch.full((H, W, 4), float("nan"), dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()            # the fill (torch's stream) before the scene's stream writes
    st = sc.render_bands(fr, 8, ids, out.data_ptr(), inplace=True, pixel_format=vx.PIXEL_RGBA32F, stats=True)
    torch.cuda.synchronize()
    img = out.cpu().numpy()
    del out
    ref = np.full((H, W, 4), np.nan, np.float32)
    acc = {}
    for j in range(8):
        _, ost = O.render(fr.params, W, H, row0=j, row_step=8 * every, threads=16, out=ref)
        for k, v in ost.as_dict().items():
            acc[k] = acc.get(k, 0) + v
    rows = [r for b in ids for r in range(8 * b, min(H, 8 * b + 8))]
    a, b = img[rows], ref[rows]
    assert not np.isnan(a).any() and not np.isnan(b).any()
    assert acc["pixels"] == len(rows) * W and acc["shadow_fetches"] > 0
    bad = int(np.count_nonzero(a.view(np.uint32) != b.view(np.uint32)))
    assert bad == 0, f"{bad} words differ from the literal march"
    g = st.as_dict()
    for k, v in acc.items():
        assert g[k] == v, (k, g[k], v)
    return rows, a


def _frames_equal_and_literal(sc, fr_default, fr_literal, W, H, O):
    """The default frame (exit tables) equals the literal frame on every pixel
    (both on the device, RGBA32F), and the literal frame's band subset equals
    the oracle's literal march, counters included."""
    import voxmap_amd as vx
    a, sa = sc.render(fr_default, stats=True)
    b, sb = sc.render(fr_literal, stats=True)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
    assert sb.shadow_fetches > sa.shadow_fetches
    rows, sub = _literal_subset(sc, fr_literal, W, H, O)
    assert np.array_equal(sub.view(np.uint32), b[rows].view(np.uint32))
    return sa, sb


def test_c5_full_size_literal_march(noise):
    """C5 (3^3-upscaled 3072x768x96 field, 3840x2160, 16-sample soft shadows,
    full quality): the default frame -- cone exit table, the first-step face-bit
    test that settles all 16 samples at once -- equals the frame marched
    without tables on every pixel, and a band subset of that frame equals the
    oracle's literal march, every word and counter."""
    import oracle
    import voxmap_amd as vx
    from voxmap_amd import presets
    grid = presets.scene_grid("s_up3")
    Z, Y, X = grid.shape
    c = presets.CONFIGS["C5"]
    kw = dict(scale=3.0, shadow_samples=16, sun_radius=0.03)
    fd = presets.camera_frame("K1", c["w"], c["h"], flags=vx.FLAG_FULL_QUALITY, **kw)
    fl = presets.camera_frame("K1", c["w"], c["h"], flags=vx.FLAG_FULL_QUALITY | vx.FLAG_NO_EXIT, **kw)
    with vx.Scene(map_bytes=grid.tobytes(), map_format=vx.FORMAT_GRID, noise_bytes=noise.tobytes(),
                  noise_format=vx.FORMAT_BIN, dims=(X, Y, Z), device=0) as sc:
        del grid
        field = sc.read_field(0)
        oct_e = [np.ascontiguousarray(sc.read_boxes(o)[..., 1:]) for o in range(8)]
        O = oracle.Oracle(field, noise, oct_e=oct_e, exit=False)
        sa, sb = _frames_equal_and_literal(sc, fd, fl, c["w"], c["h"], O)
    assert sa.shadow_rays_resolved > 0 and sb.shadow_rays_resolved == 0


def test_c3_reflect_all_full_size_literal_march(noise):
    """C3 K1 full quality + REFLECT_ALL (the general kernel, every first surface
    mirrored): exit tables vs none, and the literal march against the oracle."""
    import oracle
    import voxmap_amd as vx
    from voxmap_amd import presets
    field = vx.field_build(presets.scene_grid("s_proc"))
    f = vx.FLAG_FULL_QUALITY | vx.FLAG_REFLECT_ALL
    fd = presets.camera_frame("K1", 3840, 2160, flags=f)
    fl = presets.camera_frame("K1", 3840, 2160, flags=f | vx.FLAG_NO_EXIT)
    with vx.Scene(map_bytes=field.tobytes(), map_format=vx.FORMAT_BIN, noise_bytes=noise.tobytes(),
                  noise_format=vx.FORMAT_BIN, dims=(1024, 256, 32), device=0) as sc:
        sa, _ = _frames_equal_and_literal(sc, fd, fl, 3840, 2160, oracle.Oracle(field, noise, exit=False))
    assert sa.reflect_rays > 6_000_000


@pytest.mark.parametrize("order", [0, 0x1000], ids=["default", "general"])
def test_s_glass_c3_full_size_literal_march(noise, order):
    """S-glass C3 K1 full quality, glass in draw order -- the default (stacked
    chain in the main kernel) and VX_FLAG_GLASS_ORDER (the general kernel): the
    march runs once per blended pane; exit tables vs none, and the literal
    march against the oracle."""
    import oracle
    import voxmap_amd as vx
    from voxmap_amd import presets
    field = vx.field_build(presets.scene_grid("s_glass"))
    f = vx.FLAG_FULL_QUALITY | order
    fd = presets.camera_frame("K1", 3840, 2160, flags=f)
    fl = presets.camera_frame("K1", 3840, 2160, flags=f | vx.FLAG_NO_EXIT)
    with vx.Scene(map_bytes=field.tobytes(), map_format=vx.FORMAT_BIN, noise_bytes=noise.tobytes(),
                  noise_format=vx.FORMAT_BIN, dims=(1024, 256, 32), device=0) as sc:
        sa, _ = _frames_equal_and_literal(sc, fd, fl, 3840, 2160, oracle.Oracle(field, noise, exit=False))
    assert sa.glass_px > 100000
