"""The raster's G-buffer split on the GPU:
the device's greedy mesh per face (k_face_quads) against the oracle's, and
frames whose fragments carry the quad-relative split (the default) or the
unit-cell one (VX_FLAG_UNIT_GBUF) against the oracle in the same mode, bit for
bit, with every work counter -- on small scenes, the BASELINE C3 frame, the
stacked-glass scene S-glass and a non-default mesh CHUNK."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu(built):
    try:
        import torch
        ok = torch.cuda.is_available()
    except Exception:  # pragma: no cover
        ok = False
    if not ok:
        pytest.skip("no GPU visible")


def _scene(vx, field, noise, dims, **kw):
    X, Y, Z = dims
    return vx.Scene(map_bytes=field.tobytes(), map_format=vx.FORMAT_BIN, noise_bytes=noise.tobytes(),
                    noise_format=vx.FORMAT_BIN, dims=(X, Y, Z), device=0, **kw)


def _compare(img, ref):
    bad = int(np.count_nonzero(img.view(np.uint32) != ref.view(np.uint32)))
    if bad:
        idx = np.argwhere(img.view(np.uint32) != ref.view(np.uint32))[:5]
        raise AssertionError(f"{bad} words differ; first at {idx.tolist()}")


def _counters_equal(st, ost):
    g, o = st.as_dict(), ost.as_dict()
    for k in o:
        assert g[k] == o[k], (k, g[k], o[k])


@pytest.mark.parametrize("seed,dims,chunk", [(0, (64, 32, 16), 0), (1, (70, 40, 16), 0), (2, (96, 48, 24), 8),
                                             (3, (80, 40, 12), 40)])
def test_face_table_matches_oracle_small(noise, seed, dims, chunk):
    import oracle
    import voxmap_amd as vx
    from voxmap_amd import scenes
    field = vx.field_build(scenes.small_proc(seed, dims=dims, n_boxes=12, n_glass=4))
    with _scene(vx, field, noise, dims, mesh_chunk=chunk) as sc:
        q = sc.read_face_quads()
    ref = oracle.face_quads(field, chunk)
    assert (ref != 0xFFFF).sum() > 1000
    assert np.array_equal(q, ref)


@pytest.mark.parametrize("scene", ["s_proc", "s_glass", "s_up3"])
def test_face_table_matches_oracle_baseline(scene):
    """The BASELINE fields (C2-C4 S-proc, the stacked-glass fixture, C5's 3^3
    field with CHUNK = Z = 96), built on the device from the palette grid."""
    import oracle
    import voxmap_amd as vx
    from voxmap_amd import presets
    grid = presets.scene_grid(scene)
    Z, Y, X = grid.shape
    with vx.Scene(map_bytes=grid.tobytes(), map_format=vx.FORMAT_GRID, dims=(X, Y, Z), device=0) as sc:
        field = sc.read_field(0)
        q = sc.read_face_quads()
    ref = oracle.face_quads(field)
    assert np.array_equal(q, ref), int(np.count_nonzero(q != ref))


SMALL = [
    (5, (96, 48, 16), (48.0, 24.0, 18.0), (1.1, 0.0, 0.6)),
    (11, (128, 64, 24), (-6.0, 32.0, 9.0), (1.45, 0.0, -1.5707963267948966)),
    (13, (128, 64, 24), (64.0, 32.0, 6.0), (1.3, 0.0, 2.4)),
]


@pytest.mark.parametrize("quad", [True, False], ids=["quad", "unit"])
@pytest.mark.parametrize("seed,dims,sbj,rot", SMALL)
@pytest.mark.parametrize("flags,samples", [(0, 0), (48, 0), (48, 16), (48 | 0x80, 16), (48 | 0x100, 16)],
                         ids=["v1", "full", "soft16", "soft16_pool", "soft16_brick"])
def test_small_frames_both_splits(noise, seed, dims, sbj, rot, flags, samples, quad):
    import oracle
    import voxmap_amd as vx
    from voxmap_amd import scenes
    field = vx.field_build(scenes.small_proc(seed, dims=dims, n_boxes=16, n_glass=6))
    f = flags | (0 if quad else vx.FLAG_UNIT_GBUF)
    fr = vx.make_frame(sbj, rot, 160, 96, flags=f, shadow_samples=samples, sun_radius=0.04)
    with _scene(vx, field, noise, dims) as sc:
        img, st = sc.render(fr, stats=True)
    ref, ost = oracle.Oracle(field, noise, exit=True, quad=quad).render(fr.params, 160, 96)
    _compare(img, ref)
    _counters_equal(st, ost)


@pytest.mark.parametrize("flags", [0, 48], ids=["v1", "full"])
def test_c3_unit_split_matches_oracle(noise, flags):
    """The ABI <= 7 split on the bench's C3 frame (both kept exact)."""
    import oracle
    import voxmap_amd as vx
    from voxmap_amd import presets
    field = vx.field_build(presets.scene_grid("s_proc"))
    fr = presets.camera_frame("K1", 3840, 2160, flags=flags | vx.FLAG_UNIT_GBUF)
    with _scene(vx, field, noise, (1024, 256, 32)) as sc:
        img, st = sc.render(fr, stats=True)
    ref, ost = oracle.Oracle(field, noise, exit=True, quad=False).render(fr.params, 3840, 2160, threads=16)
    _compare(img, ref)
    _counters_equal(st, ost)


@pytest.mark.parametrize("cam,flags", [("K0", 48), ("K1", 48), ("K2", 48), ("K1", 0)])
def test_s_glass_c3_default_draw_order(noise, cam, flags):
    """S-glass (panes that stack along view rays), C3, default flags: glass in
    draw order (render.js:82-91) -- the stacked pixels' chain in the main
    kernels (EXT 0/1: glass_chain) with the GL blend stage -- every pixel and
    counter against the oracle, and the same frame and counters as the
    whole-frame general kernel (VX_FLAG_GLASS_ORDER, EXT 5) on every word."""
    import oracle
    import voxmap_amd as vx
    from voxmap_amd import presets
    field = vx.field_build(presets.scene_grid("s_glass"))
    fr = presets.camera_frame(cam, 3840, 2160, flags=flags)
    fo = presets.camera_frame(cam, 3840, 2160, flags=flags | vx.FLAG_GLASS_ORDER)
    with _scene(vx, field, noise, (1024, 256, 32)) as sc:
        img, st = sc.render(fr, stats=True)
        img_o, st_o = sc.render(fo, stats=True)
    ref, ost = oracle.Oracle(field, noise, exit=True).render(fr.params, 3840, 2160, threads=16)
    _compare(img, ref)
    _counters_equal(st, ost)
    _compare(img_o, img)
    _counters_equal(st_o, ost)
    assert st.glass_px > 100000


@pytest.mark.parametrize("cam", ["K1", "K2"])
def test_s_glass_c3_single_layer(noise, cam):
    """S-glass, C3 full quality, the single layer (VX_FLAG_GLASS_SINGLE, the
    ABI <= 8 default, kept as a diagnostic): every pixel and counter against
    the oracle."""
    import oracle
    import voxmap_amd as vx
    from voxmap_amd import presets
    grid = presets.scene_grid("s_glass")
    field = vx.field_build(grid)
    fr = presets.camera_frame(cam, 3840, 2160, flags=vx.FLAG_FULL_QUALITY | vx.FLAG_GLASS_SINGLE)
    with _scene(vx, field, noise, (1024, 256, 32)) as sc:
        img, st = sc.render(fr, stats=True)
    ref, ost = oracle.Oracle(field, noise, exit=True).render(fr.params, 3840, 2160, threads=16)
    _compare(img, ref)
    _counters_equal(st, ost)
    assert st.glass_px > 100000


def test_mesh_chunk_option(noise):
    """A scene meshed with CHUNK 16 on a Z = 32 field: the device table and the
    frames follow the option (VX scene_desc.mesh_chunk)."""
    import oracle
    import voxmap_amd as vx
    from voxmap_amd import scenes
    dims = (128, 64, 32)
    field = vx.field_build(scenes.small_proc(21, dims=dims, n_boxes=20, n_glass=6))
    fr = vx.make_frame((64.0, 32.0, 30.0), (1.1, 0.0, 0.6), 200, 120, flags=48)
    with _scene(vx, field, noise, dims, mesh_chunk=16) as sc:
        q = sc.read_face_quads()
        img, st = sc.render(fr, stats=True)
    ref_q = oracle.face_quads(field, 16)
    assert np.array_equal(q, ref_q)
    assert not np.array_equal(ref_q, oracle.face_quads(field, 0))
    ref, ost = oracle.Oracle(field, noise, exit=True, quad=ref_q, chunk=16).render(fr.params, 200, 120)
    _compare(img, ref)
    _counters_equal(st, ost)


GLASS_CASES = [
    # small S-glass scenes: hollow pavilions and screens, cameras toward -x/-y
    # (far panes' quads drawn first: both blend) and +x
    (2, (96, 64, 16), (48.0, 32.0, 20.0), (1.1, 0.0, 0.6)),
    (3, (96, 64, 16), (48.0, 32.0, 20.0), (1.2, 0.0, 2.6)),
    (4, (128, 64, 24), (64.0, 32.0, 14.0), (1.3, 0.0, -2.2)),
]


@pytest.mark.parametrize("seed,dims,sbj,rot", GLASS_CASES)
@pytest.mark.parametrize("flags,samples", [(0, 0), (48, 0), (48, 16), (48 | 0x80, 16), (48 | 0x100, 16),
                                           (0x1000, 0), (48 | 0x1000, 0), (0x2000 | 0x1000 | 32, 0), (0x2000 | 48, 0),
                                           (48 | 0x1000, 16), (48 | 0x8000, 0)],
                         ids=["v1", "full", "soft16", "soft16_pool", "soft16_brick", "general_v1", "general_full",
                              "general_reflect_all", "reflect_all", "general_soft16", "single_full"])
def test_glass_order_small(noise, seed, dims, sbj, rot, flags, samples):
    """Glass in draw order (render.js:82-91), the default -- in the main kernels
    (EXT 0-4) and in the general ones (VX_FLAG_GLASS_ORDER, REFLECT_ALL: EXT 5/6)
    -- and the single-layer diagnostic, against the oracle's restatement, every
    pixel and counter."""
    import oracle
    import voxmap_amd as vx
    from voxmap_amd import scenes
    field = vx.field_build(scenes.s_glass(seed, dims=dims, n_houses=12, n_facades=4))
    fr = vx.make_frame(sbj, rot, 200, 120, flags=flags, shadow_samples=samples, sun_radius=0.04)
    with _scene(vx, field, noise, dims) as sc:
        img, st = sc.render(fr, stats=True)
    O = oracle.Oracle(field, noise, exit=True)
    ref, ost = O.render(fr.params, 200, 120)
    _compare(img, ref)
    _counters_equal(st, ost)
    assert st.glass_px > 500


@pytest.mark.parametrize("cam", ["K1", "K2"])
def test_s_glass_c3_draw_order(noise, cam):
    """S-glass C3 full quality with glass in draw order: every pixel against the
    oracle, and (K1) the pixels that change against the single layer."""
    import oracle
    import voxmap_amd as vx
    from voxmap_amd import presets
    field = vx.field_build(presets.scene_grid("s_glass"))
    fr = presets.camera_frame(cam, 3840, 2160, flags=vx.FLAG_FULL_QUALITY | vx.FLAG_GLASS_ORDER)
    with _scene(vx, field, noise, (1024, 256, 32)) as sc:
        img, st = sc.render(fr, stats=True)
    ref, ost = oracle.Oracle(field, noise, exit=True).render(fr.params, 3840, 2160, threads=16)
    _compare(img, ref)
    _counters_equal(st, ost)


@pytest.mark.parametrize("seed,dims,sbj,rot", SMALL)
@pytest.mark.parametrize("flags", [0x2000, 0x2000 | 32, 0x2000 | 48], ids=["reflect_all", "reflect_all_rough", "full_all"])
def test_reflect_all_small(noise, seed, dims, sbj, rot, flags):
    """VX_FLAG_REFLECT_ALL: every first surface mirrors the traced scene."""
    import oracle
    import voxmap_amd as vx
    from voxmap_amd import scenes
    field = vx.field_build(scenes.small_proc(seed, dims=dims, n_boxes=16, n_glass=6))
    fr = vx.make_frame(sbj, rot, 160, 96, flags=flags)
    with _scene(vx, field, noise, dims) as sc:
        img, st = sc.render(fr, stats=True)
    ref, ost = oracle.Oracle(field, noise, exit=True).render(fr.params, 160, 96)
    _compare(img, ref)
    _counters_equal(st, ost)
    assert st.reflect_rays >= st.block_px


def test_reflect_all_c3(noise):
    """The bench's c3_reflect_all frame (full quality + REFLECT_ALL) at C3."""
    import oracle
    import voxmap_amd as vx
    from voxmap_amd import presets
    field = vx.field_build(presets.scene_grid("s_proc"))
    fr = presets.camera_frame("K1", 3840, 2160, flags=vx.FLAG_FULL_QUALITY | vx.FLAG_REFLECT_ALL)
    with _scene(vx, field, noise, (1024, 256, 32)) as sc:
        img, st = sc.render(fr, stats=True)
    ref, ost = oracle.Oracle(field, noise, exit=True).render(fr.params, 3840, 2160, threads=16)
    _compare(img, ref)
    _counters_equal(st, ost)
    assert st.reflect_rays > 6_000_000


def test_glass_more_than_eight_panes(noise):
    """Ten stacked panes, all drawn far to near (every one blends): the default
    kernels and the general ones against the oracle (no layer cap)."""
    import oracle
    import voxmap_amd as vx
    from test_quad_gbuf import _many_panes
    field = vx.field_build(_many_panes(10))
    O = oracle.Oracle(field, noise, exit=True)
    for flags in (48, 48 | 0x1000):
        fr = vx.make_frame((45.0 - 5.4, 12.2, 5.4), (1.5707, 0.0, np.pi / 2), 64, 64, flags=flags)
        with _scene(vx, field, noise, (64, 24, 12)) as sc:
            img, st = sc.render(fr, stats=True)
        ref, ost = O.render(fr.params, 64, 64)
        _compare(img, ref)
        _counters_equal(st, ost)
        assert (O.glass_layers(fr.params, 64, 64) >= 9).sum() > 400


def test_scene_without_face_table(noise, monkeypatch):
    """a field whose face table does not fit still loads (the
    allocation forced to fail); its 3D frames then need the unit-cell split
    and the single glass layer -- the only ones that read no mesh -- and it
    refuses the others with VX_EINVAL instead of rendering something else."""
    import oracle
    import voxmap_amd as vx
    from voxmap_amd import scenes
    dims = (96, 64, 16)
    field = vx.field_build(scenes.s_glass(2, dims=dims, n_houses=12, n_facades=4))
    monkeypatch.setenv("VOXMAP_TEST_NO_FACE_TABLE", "1")
    sc = _scene(vx, field, noise, dims)
    monkeypatch.delenv("VOXMAP_TEST_NO_FACE_TABLE")
    with sc:
        for flags in (48, 48 | vx.FLAG_UNIT_GBUF, 48 | vx.FLAG_GLASS_SINGLE,
                      48 | vx.FLAG_UNIT_GBUF | vx.FLAG_GLASS_SINGLE | vx.FLAG_GLASS_ORDER):
            with pytest.raises(vx.VoxmapError) as e:
                sc.render(vx.make_frame((48.0, 32.0, 20.0), (1.1, 0.0, 0.6), 64, 48, flags=flags))
            assert e.value.code == -1 and "face table" in str(e.value)
        with pytest.raises(vx.VoxmapError):
            sc.read_face_quads()
        fr = vx.make_frame((48.0, 32.0, 20.0), (1.1, 0.0, 0.6), 200, 120,
                           flags=48 | vx.FLAG_UNIT_GBUF | vx.FLAG_GLASS_SINGLE)
        img, st = sc.render(fr, stats=True)
    ref, ost = oracle.Oracle(field, noise, exit=True, quad=False).render(fr.params, 200, 120)
    _compare(img, ref)
    _counters_equal(st, ost)
    assert st.glass_px > 500
