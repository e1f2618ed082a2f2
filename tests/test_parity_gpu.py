"""Parity of the HIP path (libvoxmap_hip.so on device 0) with the scalar oracle.

Bar: bit-exact fp32 (DESIGN.md §5 numerical contract), identical work
counters, identical A channel, on EVERY pixel -- including the BASELINE sizes
(C2 1920x1080 for cameras K0-K2, C3 3840x2160 v1 and full quality = the bench's
own frame, C4 7680x4320 through the 8-rank band lists, C5 3840x2160 on the
3^3-upscaled field with 16-sample soft shadows): the oracle renders a C3 frame
in about a quarter second on the box's 16 cores.  Plus size-independent
properties (RGBA8 == quantised RGBA32F, tiles == frame, bands == frame).
"""
import math

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _torch_gpu():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:  # pragma: no cover
        return False


@pytest.fixture(scope="module", autouse=True)
def _need_gpu(built):
    if not _torch_gpu():
        pytest.skip("no GPU visible")


def _scene(vx, field, noise, dims):
    X, Y, Z = dims
    return vx.Scene(map_bytes=field.tobytes(), map_format=vx.FORMAT_BIN, noise_bytes=noise.tobytes(),
                    noise_format=vx.FORMAT_BIN, dims=(X, Y, Z), device=0)


def _vis(b):
    """The traversal's colour: meshed palette indices 1..21 (sdf.cpp:284), else 0 (include/voxmap.h)."""
    return np.where((b >= 1) & (b <= 21), b, 0).astype(np.uint8)


def _diff(a, b):
    return int(np.count_nonzero(a.view(np.uint32) != b.view(np.uint32)))


def _counters_equal(st, ost, keys=None):
    g, o = st.as_dict(), ost.as_dict()
    for k in keys or o:
        assert g[k] == o[k], (k, g[k], o[k])


def _compare(img, ref, rows=None):
    if rows is not None:
        img, ref = img[rows], ref[rows]
    bad = _diff(img, ref)
    if bad:
        idx = np.argwhere(img.view(np.uint32) != ref.view(np.uint32))[:5]
        rel = np.max(np.abs(img - ref) / np.maximum(np.abs(ref), 1e-6))
        raise AssertionError(f"{bad} words differ (max rel {rel:.3g}); first at {idx.tolist()}")


SMALL = [
    # (scene seed, dims, sbj, rot)
    (5, (96, 48, 16), (48.0, 24.0, 18.0), (1.1, 0.0, 0.6)),
    (7, (96, 48, 16), (48.0, 24.0, 40.0), (1e-4, 0.0, -0.002)),
    (11, (128, 64, 24), (-6.0, 32.0, 9.0), (1.45, 0.0, -math.pi / 2)),
    (13, (128, 64, 24), (64.0, 32.0, 6.0), (1.3, 0.0, 2.4)),      # camera inside the grid
]


@pytest.mark.parametrize("seed,dims,sbj,rot", SMALL)
def test_small_frames_bit_exact(seed, dims, sbj, rot, noise):
    import oracle
    import voxmap_amd as vx
    from voxmap_amd import scenes
    grid = scenes.small_proc(seed, dims=dims, n_boxes=16, n_glass=6)
    field = vx.field_build(grid)
    fr = vx.make_frame(sbj, rot, 160, 96)
    with _scene(vx, field, noise, dims) as sc:
        dev_field = sc.read_field()
        img, st = sc.render(fr, stats=True)
    ref, ost = oracle.Oracle(dev_field, noise, exit=True).render(fr.params, 160, 96)
    _compare(img, ref)
    g, o = st.as_dict(), ost.as_dict()
    for k in o:
        assert g[k] == o[k], (k, g[k], o[k])
    assert st.primary_cap_hits == 0


@pytest.mark.parametrize("octant", range(8))
def test_field_octant_copies_match_oracle(noise, octant):
    import oracle
    import voxmap_amd as vx
    from voxmap_amd import scenes
    dims = (160, 72, 20)
    field = vx.field_build(scenes.small_proc(17, dims=dims, n_boxes=24, n_glass=4))
    with _scene(vx, field, noise, dims) as sc:
        dev = sc.read_field(octant)
        box = sc.read_boxes(octant)
    assert np.array_equal(dev[..., :3], field[..., :3])
    assert np.array_equal(dev[..., 3], oracle.field_octant(field, octant))
    assert np.array_equal(box[..., 0], _vis(field[..., 2]))
    assert np.array_equal(box[..., 1:], oracle.field_box(field, octant))


@pytest.mark.parametrize("octant", [0, 3, 5])
def test_box_extents_full_scene_match_oracle(octant):
    """Device traversal boxes (k_oct_box: prefix sums + bisection) == the
    oracle's vxo_field_box on the BASELINE 1024x256x32 field, and min(e) is
    the octant's air cube (vxo_field_octant)."""
    import oracle
    import voxmap_amd as vx
    from voxmap_amd import presets
    grid = presets.scene_grid("s_proc")
    Z, Y, X = grid.shape
    with vx.Scene(map_bytes=grid.tobytes(), map_format=vx.FORMAT_GRID, dims=(X, Y, Z), device=0) as sc:
        field = sc.read_field(0)
        box = sc.read_boxes(octant)
    r = oracle.field_octant(field, octant)
    e = oracle.field_box(field, octant, r_cube=r)
    assert np.array_equal(box[..., 0], _vis(field[..., 2]))
    assert np.array_equal(box[..., 1:], e)
    assert np.array_equal(e.min(axis=3), r)


@pytest.fixture(scope="module")
def full_scene(noise):
    import voxmap_amd as vx
    from voxmap_amd import presets
    field = vx.field_build(presets.scene_grid("s_proc"))
    sc = _scene(vx, field, noise, (1024, 256, 32))
    yield sc, sc.read_field()
    sc.close()


@pytest.mark.parametrize("cfg,cam", [("C2", "K0"), ("C2", "K1"), ("C2", "K2"), ("C3", "K1")])
def test_baseline_sizes_full_frame(full_scene, noise, cfg, cam):
    """BASELINE C2 (every camera) and C3, the reference's v1 shading: every pixel
    and every work counter against the oracle."""
    import oracle
    from voxmap_amd import presets
    sc, dev_field = full_scene
    c = presets.CONFIGS[cfg]
    fr = presets.camera_frame(cam, c["w"], c["h"])
    img, st = sc.render(fr, stats=True)
    ref, ost = oracle.Oracle(dev_field, noise, exit=True).render(fr.params, c["w"], c["h"], threads=16)
    _compare(img, ref)
    _counters_equal(st, ost)
    assert st.primary_cap_hits == 0
    assert st.pixels == c["w"] * c["h"]


@pytest.mark.parametrize("w,h", [(640, 360), (333, 77), (1000, 601)])
def test_rgba8_is_quantised_rgba32f(full_scene, w, h):
    """The RGBA8 store goes through LDS (32x8-pixel blocks written as whole
    rows); ragged sizes leave partial blocks at the right and bottom edges."""
    import voxmap_amd as vx
    from voxmap_amd import presets
    sc, _ = full_scene
    fr = presets.camera_frame("K1", w, h, flags=vx.FLAG_FULL_QUALITY)
    f32, _ = sc.render(fr)
    u8, _ = sc.render(fr, pixel_format=vx.PIXEL_RGBA8)
    expect = (np.clip(f32, 0, 1) * np.float32(255) + np.float32(0.5)).astype(np.uint8)
    assert np.array_equal(u8, expect)


@pytest.mark.parametrize("cam", ["K0", "K1", "K2"])
@pytest.mark.parametrize("flags,samples", [(0, 0), (0x30, 0), (0x30, 4)])
def test_fp32_and_integer_primary_index_agree(full_scene, cam, flags, samples):
    """The fp32 x/y primary index (chosen by vx_render where exact, as on this
    field) and the integer one (VX_FLAG_INT_INDEX) give the same frame and
    counters; the oracle rows above pin the fp32 path, the C5 rows (6.7 GB of
    copies: integer path) the other."""
    import voxmap_amd as vx
    from voxmap_amd import presets
    sc, _ = full_scene
    kw = dict(shadow_samples=samples, sun_radius=0.03 if samples > 1 else 0.0)
    a, sa = sc.render(presets.camera_frame(cam, 960, 540, flags=flags, **kw), stats=True)
    b, sb = sc.render(presets.camera_frame(cam, 960, 540, flags=flags | vx.FLAG_INT_INDEX, **kw), stats=True)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
    assert sa.as_dict() | {"kernel_ms": 0} == sb.as_dict() | {"kernel_ms": 0}


@pytest.mark.parametrize("flags,samples", [(0, 0), (0x30, 0), (0x30, 4)])
def test_tiles_and_detile_equal_full_frame(full_scene, flags, samples):
    import torch
    import voxmap_amd as vx
    from voxmap_amd import presets
    sc, _ = full_scene
    w, h, ts = 1000, 600, 64            # ragged: w, h not multiples of the tile
    fr = presets.camera_frame("K1", w, h, flags=flags, shadow_samples=samples, sun_radius=0.03)
    full, _ = sc.render(fr, pixel_format=vx.PIXEL_RGBA8)
    tx, ty = -(-w // ts), -(-h // ts)
    ids = list(range(tx * ty))[::-1]    # any order
    tiles = torch.empty(len(ids) * ts * ts * 4, dtype=torch.uint8, device="cuda:0")
    frame = torch.zeros(h * w * 4, dtype=torch.uint8, device="cuda:0")
    torch.cuda.synchronize()            # the fill (torch's stream) before the scene's stream writes
    sc.render_tiles(fr, ts, ids, tiles.data_ptr())
    sc.detile(w, h, ts, ids, tiles.data_ptr(), frame.data_ptr())
    torch.cuda.synchronize()
    assert np.array_equal(frame.cpu().numpy().reshape(h, w, 4), full)


@pytest.mark.parametrize("case", ["sun_axis_zero", "sun_below", "quality0", "no_shadow", "no_ao", "no_clouds",
                                  "short_budget", "primary_only", "sun_tiny_component"])
def test_edge_params(noise, case):
    import oracle
    import voxmap_amd as vx
    from voxmap_amd import scenes
    dims = (96, 48, 16)
    grid = scenes.small_proc(21, dims=dims, n_boxes=14, n_glass=4)
    field = vx.field_build(grid)
    kw = {}
    if case == "sun_axis_zero":
        kw["sun"] = (0.6, 0.0, 0.8)          # 0*inf = NaN path of march() (render.frag:94-105)
    elif case == "sun_below":
        kw["sun"] = (0.3, 0.2, -0.93)
    elif case == "quality0":
        kw["quality"] = 0
    elif case == "no_shadow":
        kw["flags"] = vx.FLAG_NO_SHADOW
    elif case == "no_ao":
        kw["flags"] = vx.FLAG_NO_AO
    elif case == "no_clouds":
        kw["flags"] = vx.FLAG_NO_CLOUDS
    elif case == "short_budget":
        kw["max_shadow_steps"] = 5
    elif case == "primary_only":
        kw["flags"] = vx.FLAG_PRIMARY_ONLY
    elif case == "sun_tiny_component":
        kw["sun"] = (0.8, 1e-4, 0.6)         # below the fast path's 2^-10 bound: literal march
    fr = vx.make_frame((48.0, 24.0, 18.0), (1.1, 0.0, 0.6), 128, 80, **kw)
    with _scene(vx, field, noise, dims) as sc:
        dev_field = sc.read_field()
        img, st = sc.render(fr, stats=True)
    ref, ost = oracle.Oracle(dev_field, noise, exit=True).render(fr.params, 128, 80)
    _compare(img, ref)
    assert st.shadow_fetches == ost.shadow_fetches


def test_campus_scene(noise):
    import oracle
    import voxmap_amd as vx
    from voxmap_amd import presets, scenes
    field = vx.field_build(scenes.s_campus())
    fr = presets.camera_frame("K1", 480, 270)
    with _scene(vx, field, noise, (1024, 256, 32)) as sc:
        dev_field = sc.read_field()
        img, _ = sc.render(fr)
    ref, _ = oracle.Oracle(dev_field, noise, exit=True).render(fr.params, 480, 270, threads=16)
    _compare(img, ref)


# ---- extensions: REFLECT, ROUGH, soft shadows -------------------
EXT_CASES = {
    "reflect": dict(flags=0x10),
    "rough": dict(flags=0x20),
    "full_quality": dict(flags=0x30),
    "soft8": dict(shadow_samples=8, sun_radius=0.05),
    "soft16_full": dict(flags=0x30, shadow_samples=16, sun_radius=0.04),
    "soft_sun_low": dict(shadow_samples=6, sun_radius=0.3, sun=(0.9, 0.3, 0.05)),   # samples below the horizon
    "soft_axis_zero": dict(shadow_samples=4, sun_radius=0.0, sun=(0.6, 0.0, 0.8)),  # literal march per sample
    "full_no_ao_no_clouds": dict(flags=0x30 | 0x2 | 0x4),
    # VX_FLAG_SOFT_POOL (0x80): the same samples marched by the pooled wave pass
    "soft8_pool": dict(flags=0x80, shadow_samples=8, sun_radius=0.05),
    "soft6_pool": dict(flags=0x80, shadow_samples=6, sun_radius=0.05),            # 8-lane groups, 2 idle lanes
    "soft16_full_pool": dict(flags=0x30 | 0x80, shadow_samples=16, sun_radius=0.04),
    "soft_sun_low_pool": dict(flags=0x80, shadow_samples=6, sun_radius=0.3, sun=(0.9, 0.3, 0.05)),  # mixed: falls back
    # VX_FLAG_SOFT_BRICK (0x100): pooled + LDS 8^3 brick staging
    "soft16_brick": dict(flags=0x100, shadow_samples=16, sun_radius=0.05),
    "soft12_full_brick": dict(flags=0x30 | 0x100, shadow_samples=12, sun_radius=0.04),
    "soft16_brick_sun_neg": dict(flags=0x100, shadow_samples=16, sun_radius=0.05, sun=(-0.5, -0.6, 0.62)),
}


@pytest.mark.parametrize("case", list(EXT_CASES))
@pytest.mark.parametrize("seed,dims,sbj,rot", SMALL[:2] + SMALL[3:])
def test_extensions_bit_exact(seed, dims, sbj, rot, noise, case):
    import oracle
    import voxmap_amd as vx
    from voxmap_amd import scenes
    grid = scenes.small_proc(seed, dims=dims, n_boxes=16, n_glass=10)
    field = vx.field_build(grid)
    fr = vx.make_frame(sbj, rot, 160, 96, **EXT_CASES[case])
    with _scene(vx, field, noise, dims) as sc:
        dev_field = sc.read_field()
        img, st = sc.render(fr, stats=True)
    ref, ost = oracle.Oracle(dev_field, noise, exit=True).render(fr.params, 160, 96)
    _compare(img, ref)
    g, o = st.as_dict(), ost.as_dict()
    for k in o:
        assert g[k] == o[k], (k, g[k], o[k])
    assert st.primary_cap_hits == 0


@pytest.mark.parametrize("case", ["soft8", "soft8_pool", "soft6_pool", "soft16_brick", "soft12_full_brick"])
@pytest.mark.parametrize("w,h", [(157, 93), (100, 70)])
def test_soft_shadow_paths_at_ragged_sizes(noise, case, w, h):
    """Frames whose right and bottom waves are partly off the frame (w, h not
    multiples of 8): the pooled pass deals fragment x sample pairs over all 64
    lanes, so off-frame lanes must still march for the others, stage their brick
    rows and count nothing of their own."""
    import oracle
    import voxmap_amd as vx
    from voxmap_amd import scenes
    seed, dims, sbj, rot = SMALL[0]
    field = vx.field_build(scenes.small_proc(seed, dims=dims, n_boxes=16, n_glass=10))
    fr = vx.make_frame(sbj, rot, w, h, **EXT_CASES[case])
    with _scene(vx, field, noise, dims) as sc:
        dev_field = sc.read_field()
        img, st = sc.render(fr, stats=True)
    ref, ost = oracle.Oracle(dev_field, noise, exit=True).render(fr.params, w, h)
    _compare(img, ref)
    _counters_equal(st, ost)


@pytest.mark.parametrize("cfg,cam,kw", [
    ("C3", "K1", dict(flags=0x30)),                                   # BASELINE C3 "full quality": the bench frame
    ("C2", "K2", dict(flags=0x30, shadow_samples=4, sun_radius=0.03)),
])
def test_extensions_baseline_full_frame(full_scene, noise, cfg, cam, kw):
    """Full quality (REFLECT + ROUGH) at the BASELINE sizes, every pixel and
    counter; the C3 case is the bench's exact frame, also checked in the RGBA8
    format the bench renders (== the oracle quantised)."""
    import oracle
    import voxmap_amd as vx
    from voxmap_amd import presets
    sc, dev_field = full_scene
    c = presets.CONFIGS[cfg]
    fr = presets.camera_frame(cam, c["w"], c["h"], **kw)
    img, st = sc.render(fr, stats=True)
    ref, ost = oracle.Oracle(dev_field, noise, exit=True).render(fr.params, c["w"], c["h"], threads=16)
    _compare(img, ref)
    _counters_equal(st, ost)
    assert st.primary_cap_hits == 0
    assert st.reflect_rays == st.glass_px
    if cfg == "C3":
        img8, _ = sc.render(fr, pixel_format=vx.PIXEL_RGBA8)
        q = (np.clip(ref, 0, 1) * np.float32(255) + np.float32(0.5)).astype(np.uint8)
        assert np.array_equal(img8, q)


# ---- f-1: the distance field built on the GPU ----------------------------------
@pytest.mark.parametrize("name", ["small_a", "small_b", "tall", "s_proc", "s_campus", "s_up3"])
def test_gpu_field_build_equals_host(name):
    """vx_field_build_gpu (plane-parallel on the device) == vx_field_build (host
    restatement, itself checked against the literal serial oracle): every byte,
    up to the C5 3072x768x96 field."""
    import voxmap_amd as vx
    from voxmap_amd import presets, scenes
    if name == "small_a":
        grid = scenes.small_proc(3, dims=(96, 48, 16), n_boxes=16, n_glass=4)
    elif name == "small_b":
        grid = scenes.small_proc(4, dims=(40, 72, 24), n_boxes=10, n_glass=2)
    elif name == "tall":          # Z > Y: plane-0 shells clipped by Y
        grid = scenes.small_proc(9, dims=(33, 12, 40), n_boxes=6, n_glass=1)
    else:
        grid = presets.scene_grid(name)
    want = vx.field_build(grid)
    got = vx.field_build_gpu(grid)
    assert np.array_equal(got, want), int(np.count_nonzero(got != want))


def test_scene_from_grid_equals_scene_from_field(noise):
    import voxmap_amd as vx
    from voxmap_amd import scenes
    dims = (96, 48, 16)
    grid = scenes.small_proc(12, dims=dims, n_boxes=14, n_glass=5)
    field = vx.field_build(grid)
    with _scene(vx, field, noise, dims) as a, vx.Scene(map_bytes=grid.tobytes(), map_format=vx.FORMAT_GRID,
                                                     noise_bytes=noise.tobytes(), noise_format=vx.FORMAT_BIN,
                                                     dims=dims, device=0) as b:
        for o in (0, 3, 7):
            assert np.array_equal(a.read_field(o), b.read_field(o))
        fr = vx.make_frame((48.0, 24.0, 18.0), (1.1, 0.0, 0.6), 64, 48, flags=vx.FLAG_FULL_QUALITY)
        ia, _ = a.render(fr)
        ib, _ = b.render(fr)
    assert np.array_equal(ia.view(np.uint32), ib.view(np.uint32))


@pytest.mark.timeout(900)
def test_c5_full_frame_soft_shadows_full_quality(noise):
    """BASELINE C5: 3^3-upscaled 3072x768x96 field, 3840x2160, 16-sample soft
    shadows + full quality, every pixel and counter against the oracle.  The
    primary traversal of the octant most pixels look into runs on boxes the
    ORACLE computes at this size (vxo_field_octant + vxo_field_box over the
    226 M cells), so those pixels are checked independently of the device's
    field preparation; the other octants take the device's boxes, themselves
    checked against the oracle on the 1024x256x32 field above."""
    import oracle
    import voxmap_amd as vx
    from voxmap_amd import presets
    grid = presets.scene_grid("s_up3")
    Z, Y, X = grid.shape
    c = presets.CONFIGS["C5"]
    fr = presets.camera_frame("K1", c["w"], c["h"], scale=3.0, flags=vx.FLAG_FULL_QUALITY, shadow_samples=16,
                              sun_radius=0.03)
    with vx.Scene(map_bytes=grid.tobytes(), map_format=vx.FORMAT_GRID, noise_bytes=noise.tobytes(),
                  noise_format=vx.FORMAT_BIN, dims=(X, Y, Z), device=0) as sc:
        img, st = sc.render(fr, stats=True)
        field = sc.read_field(0)
        oct_e = [np.ascontiguousarray(sc.read_boxes(o)[..., 1:]) for o in range(8)]
    del grid
    import ctypes as C
    counts = np.zeros(8, np.int64)                   # octant census of the frame's view rays
    d = (C.c_float * 3)()
    for py in range(0, c["h"], 8):
        for px in range(0, c["w"], 8):
            oracle.lib().vxo_pixel_dir(C.addressof(fr.params), c["w"], c["h"], px, py, d)
            counts[int(d[0] < 0) | (int(d[1] < 0) << 1) | (int(d[2] < 0) << 2)] += 1
    main = int(np.argmax(counts))
    r = oracle.field_octant(field, main)
    own = oracle.field_box(field, main, r_cube=r)
    assert np.array_equal(own, oct_e[main])          # the device's boxes of that octant, at the C5 size
    oct_e[main] = own
    ref, ost = oracle.Oracle(field, noise, oct_e=oct_e, exit=True).render(fr.params, c["w"], c["h"], threads=16)
    _compare(img, ref)
    _counters_equal(st, ost)
    assert st.primary_cap_hits == 0


def test_soft_pool_equals_per_sample_march(noise):
    """VX_FLAG_SOFT_POOL and VX_FLAG_SOFT_BRICK at C5 (3^3 field, 16 samples,
    full quality): the pooled wave march, with and without LDS brick staging,
    gives the same RGBA8 frame and the same work counters as the per-sample
    loop, on the whole 3840x2160 frame.  The brick march reads no doom table
    (DESIGN.md §3 "Doom table"): its counters are the per-sample loop's with
    VX_FLAG_NO_DOOM."""
    import torch
    import voxmap_amd as vx
    from voxmap_amd import presets
    grid = presets.scene_grid("s_up3")
    Z, Y, X = grid.shape
    c = presets.CONFIGS["C5"]
    outs, sts = [], []
    with vx.Scene(map_bytes=grid.tobytes(), map_format=vx.FORMAT_GRID, noise_bytes=noise.tobytes(),
                  noise_format=vx.FORMAT_BIN, dims=(X, Y, Z), device=0) as sc:
        for extra in (0, vx.FLAG_SOFT_POOL, vx.FLAG_SOFT_BRICK, vx.FLAG_NO_DOOM):
            fr = presets.camera_frame("K1", c["w"], c["h"], scale=3.0, flags=vx.FLAG_FULL_QUALITY | extra,
                                      shadow_samples=16, sun_radius=0.03)
            out = torch.zeros(c["w"] * c["h"] * 4, dtype=torch.uint8, device="cuda:0")
            torch.cuda.synchronize()         # the fill (torch's stream) before the scene's stream writes
            sts.append(sc.render_device(fr, out.data_ptr(), pixel_format=vx.PIXEL_RGBA8, stats=True))
            torch.cuda.synchronize()
            outs.append(out.cpu().numpy())
    for i in (1, 2, 3):
        assert np.array_equal(outs[0], outs[i]), i
    for i, j in ((0, 1), (3, 2)):
        a, b = sts[i].as_dict(), sts[j].as_dict()
        for k in ("shadow_rays", "shadow_fetches", "primary_fetches", "ao_samples", "alg_bytes"):
            assert a[k] == b[k], (i, k, a[k], b[k])


# ---- the reference's map.bin air encoding ------------------
def test_air_b22_and_b0_render_identically(noise, tmp_path):
    """map.bin from sdf.cpp writes air as B = pal_size = 22 (sdf.cpp:229-233,
    466-468); a pre-remap grid has 0.  Both must give identical frames and
    identical work counters (primary fetches: the traversal boxes ignore the
    encoding) -- through FORMAT_BIN here and through a .blob in vxrender
    (tests/test_cli.py) -- and equal the oracle."""
    import oracle
    import voxmap_amd as vx
    from voxmap_amd import scenes
    dims = (128, 64, 24)
    grid = scenes.small_proc(11, dims=dims, n_boxes=16, n_glass=12)
    f22 = vx.field_build(grid)
    assert (f22[..., 2][grid == 0] == 22).all()
    f0 = f22.copy()
    f0[..., 2][grid == 0] = 0
    fr = vx.make_frame((64.0, 32.0, 14.0), (1.2, 0.0, 2.0), 160, 96, flags=vx.FLAG_FULL_QUALITY)
    imgs, sts = [], []
    for f in (f22, f0):
        with _scene(vx, f, noise, dims) as sc:
            img, st = sc.render(fr, stats=True)
            assert np.array_equal(sc.read_field()[..., :3], f[..., :3])     # B read back as uploaded
        imgs.append(img)
        sts.append(st.as_dict() | {"kernel_ms": 0})
    assert np.array_equal(imgs[0].view(np.uint32), imgs[1].view(np.uint32))
    assert sts[0] == sts[1] and sts[0]["glass_px"] > 100
    ref, _ = oracle.Oracle(f22, noise, exit=True).render(fr.params, 160, 96)
    _compare(imgs[0], ref)


def test_hand_edited_map_with_large_radii_uses_the_checked_march(noise):
    """A map.bin whose R/G values exceed Z (not produced by sdf.cpp) must not
    take the padded int8 march (its border assumes steps <= Z + 1 cells):
    vx_scene_create falls back to the bounds-checked march, equal to the oracle."""
    import oracle
    import voxmap_amd as vx
    from voxmap_amd import scenes
    dims = (96, 48, 16)
    field = vx.field_build(scenes.small_proc(21, dims=dims, n_boxes=14, n_glass=4))
    air = field[..., 0] > 0
    field[..., 0][air] = np.minimum(255, field[..., 0][air].astype(int) * 9).astype(np.uint8)   # R up to 144+
    field[5, 10, 10, 0] = 200
    fr = vx.make_frame((48.0, 24.0, 18.0), (1.1, 0.0, 0.6), 128, 80)
    with _scene(vx, field, noise, dims) as sc:
        img, st = sc.render(fr, stats=True)
    ref, ost = oracle.Oracle(field, noise, exit=True).render(fr.params, 128, 80)
    _compare(img, ref)
    assert st.shadow_fetches == ost.shadow_fetches


# ---- the multi-GPU unit: full-width bands (vx_render_bands, vx_mgpu_*) -----------
@pytest.mark.parametrize("fmt", ["rgba8", "rgba32f"])
def test_bands_inplace_and_compact_equal_full_frame(full_scene, fmt):
    import torch
    import voxmap_amd as vx
    from voxmap_amd import presets
    sc, _ = full_scene
    w, h, br = 1000, 601, 64                 # ragged: last band 25 rows, w not a multiple of 32
    pf = vx.PIXEL_RGBA8 if fmt == "rgba8" else vx.PIXEL_RGBA32F
    ch, dt = (4, torch.uint8) if fmt == "rgba8" else (4, torch.float32)
    fr = presets.camera_frame("K1", w, h, flags=vx.FLAG_FULL_QUALITY)
    full, _ = sc.render(fr, pixel_format=pf)
    nb = -(-h // br)
    frame = torch.full((h, w, ch), 7, dtype=dt, device="cuda:0")
    torch.cuda.synchronize()                 # the fill (torch's stream) before the scene's stream writes
    for world in (3,):
        for r in range(world):                        # every rank's deal, in place in one frame
            sc.render_bands(fr, br, vx.mgpu_bands(h, br, world, r), frame.data_ptr(), inplace=True, pixel_format=pf)
    torch.cuda.synchronize()
    got = frame.cpu().numpy()
    assert np.array_equal(got.view(np.uint8), full.view(np.uint8))
    ids = list(range(nb))[::-1]                       # compact, any order
    comp = torch.zeros((nb * br, w, ch), dtype=dt, device="cuda:0")
    torch.cuda.synchronize()
    sc.render_bands(fr, br, ids, comp.data_ptr(), inplace=False, pixel_format=pf)
    torch.cuda.synchronize()
    comp = comp.cpu().numpy()
    for k, b in enumerate(ids):
        rows = min(br, h - b * br)
        assert np.array_equal(comp[k * br:k * br + rows].view(np.uint8), full[b * br:b * br + rows].view(np.uint8))


def test_mgpu_single_rank_equals_full_frame(full_scene):
    """vx_mgpu_* at one rank (the one GPU of this box): communicator creation,
    the band render in place, the (empty) gather; N > 1 runs in bench.py."""
    import torch
    import voxmap_amd as vx
    from voxmap_amd import presets
    sc, _ = full_scene
    w, h = 960, 544
    fr = presets.camera_frame("K2", w, h, flags=vx.FLAG_FULL_QUALITY)
    full, st_full = sc.render(fr, pixel_format=vx.PIXEL_RGBA8, stats=True)
    mg = vx.MultiGPU(sc, vx.mgpu_unique_id(), 1, 0)
    try:
        frame = torch.zeros((h, w, 4), dtype=torch.uint8, device="cuda:0")
        torch.cuda.synchronize()                     # the fill before the scene's stream writes
        st = mg.render(fr, 64, frame.data_ptr(), stats=True)
        mg.gather(w, h, 64, frame.data_ptr())        # the gather step alone (bench's split timing)
        torch.cuda.synchronize()
        with pytest.raises(RuntimeError):
            mg.gather(w, h, 60, frame.data_ptr())    # band rows must be a multiple of 8
    finally:
        mg.close()
    assert np.array_equal(frame.cpu().numpy(), full)
    assert st.pixels == w * h and st.shadow_fetches == st_full.shadow_fetches


# ---- BASELINE configs never exercised in round 1 -----------------
def test_c1_primary_only_every_pixel(noise):
    """C1: 256x256 primary-ray-only render of the 1024x256x32 field (camera K0),
    every pixel against the oracle (and its visibility counters)."""
    import oracle
    import voxmap_amd as vx
    from voxmap_amd import presets
    c = presets.CONFIGS["C1"]
    field = vx.field_build(presets.scene_grid("s_proc"))
    fr = presets.camera_frame(c["camera"], c["w"], c["h"], flags=vx.FLAG_PRIMARY_ONLY)
    with _scene(vx, field, noise, (1024, 256, 32)) as sc:
        img, st = sc.render(fr, stats=True)
    ref, ost = oracle.Oracle(field, noise, exit=True).render(fr.params, c["w"], c["h"])
    _compare(img, ref)
    for k in ("pixels", "sky_px", "block_px", "glass_px", "primary_fetches"):
        assert getattr(st, k) == getattr(ost, k), k
    assert st.shadow_rays == 0 and st.ao_samples == 0


def test_c4_full_frame_as_eight_rank_band_lists(full_scene, noise):
    """C4: 7680x4320 full quality rendered as the 8 ranks' band lists (in place,
    the vx_mgpu deal), in RGBA32F, every pixel against the oracle; and the same
    lists in RGBA8 == vx_render of the whole frame."""
    import oracle
    import torch
    import voxmap_amd as vx
    from voxmap_amd import presets
    sc, dev_field = full_scene
    c = presets.CONFIGS["C4"]
    w, h, br = c["w"], c["h"], 64
    fr = presets.camera_frame(c["camera"], w, h, flags=vx.FLAG_FULL_QUALITY)
    frame = torch.full((h, w, 4), float("nan"), dtype=torch.float32, device="cuda:0")
    torch.cuda.synchronize()                 # the fill (torch's stream) before the scene's stream writes
    for r in range(8):
        sc.render_bands(fr, br, vx.mgpu_bands(h, br, 8, r), frame.data_ptr(), inplace=True,
                        pixel_format=vx.PIXEL_RGBA32F)
    torch.cuda.synchronize()
    img = frame.cpu().numpy()
    del frame
    ref, _ = oracle.Oracle(dev_field, noise, exit=True).render(fr.params, w, h, threads=16)
    _compare(img, ref)
    del img, ref
    whole = torch.empty((h, w, 4), dtype=torch.uint8, device="cuda:0")
    sc.render_device(fr, whole.data_ptr(), pixel_format=vx.PIXEL_RGBA8)
    f8 = torch.zeros((h, w, 4), dtype=torch.uint8, device="cuda:0")
    torch.cuda.synchronize()
    for r in range(8):
        sc.render_bands(fr, br, vx.mgpu_bands(h, br, 8, r), f8.data_ptr(), inplace=True)
    torch.cuda.synchronize()
    assert torch.equal(f8, whole)


# ---- 2D mode (u_quality = 0: the vertex2d footprint mesh, render.js:278,287) ----------
@pytest.mark.parametrize("case", ["glass_scene", "campus_K0", "camera_below", "grazing"])
def test_2d_mode_bit_exact(noise, case):
    import oracle
    import voxmap_amd as vx
    from voxmap_amd import presets, scenes
    if case == "campus_K0":
        dims = (1024, 256, 32)
        grid = scenes.s_campus()
        fr = presets.camera_frame("K0", 512, 256, quality=0)
    else:
        dims = (128, 64, 24)
        grid = scenes.small_proc(11, dims=dims, n_boxes=16, n_glass=40)
        sbj, rot = {"glass_scene": ((64.0, 32.0, 30.0), (0.6, 0.0, 0.4)),
                    "camera_below": ((64.0, 32.0, -20.0), (2.5, 0.0, 0.0)),
                    "grazing": ((-10.0, 32.0, 6.0), (1.5, 0.0, -math.pi / 2))}[case]
        fr = vx.make_frame(sbj, rot, 160, 96, quality=0)
    field = vx.field_build(grid)
    with _scene(vx, field, noise, dims) as sc:
        img, st = sc.render(fr, stats=True)
        assert sc.vertex2d() == vx.vertex2d(field)          # the scene's 2D mesh = the host restatement
    ref, ost = oracle.Oracle(field, noise, exit=True).render(fr.params, fr.width, fr.height)
    _compare(img, ref)
    for k in ("pixels", "sky_px", "block_px", "glass_px", "primary_fetches"):
        assert getattr(st, k) == getattr(ost, k), k
    if case == "glass_scene":
        assert st.glass_px > 50 and st.block_px > 1000
    if case == "camera_below":
        assert st.sky_px == st.pixels                       # culled from below: the clear colour only
