"""The sun doom table on the GPU (DESIGN.md §3 "Doom table"): launch_sun_doom
builds it into the frame's cone copy and the padded march ends a ray unlit at
a doomed cell when the budget rule allows (else it goes on from the cell's
texel).  Frames equal the oracle's and the frames without the table
(VX_FLAG_NO_DOOM) bit for bit; the shadow fetch counters equal the oracle's
with and without the table (so the device table and the march's stopping rule
agree with vxo_field_doom and march_ex landing by landing in count); at the
bench scenes (S-proc, S-glass, C5's 3^3 field) with C5's 16 soft samples frames
are identical with and without the table and the table removes shadow fetches.
Hard and soft shadows read the table."""
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


def _sun(el_deg, az_deg):
    el, az = math.radians(el_deg), math.radians(az_deg)
    return (math.cos(el) * math.cos(az), math.cos(el) * math.sin(az), math.sin(el))


# soft shadows, and hard shadows (one sample)
SUNS = [(33, 30, 0.02, 4), (40, 120, 0.02, 4), (60, 210, 0.03, 8), (20, 300, 0.02, 2), (15, 45, 0.01, 4),
        (45, 160, 0.05, 8), (25, 250, 0.04, 16), (15, 45, 0.0, 1)]


@pytest.fixture(scope="module")
def small(noise):
    import voxmap_amd as vx
    from voxmap_amd import scenes
    dims = (96, 64, 40)
    field = vx.field_build(scenes.small_proc(31, dims=dims, n_boxes=30, n_glass=5))
    sc = vx.Scene(map_bytes=field.tobytes(), map_format=vx.FORMAT_BIN, noise_bytes=noise.tobytes(),
                  noise_format=vx.FORMAT_BIN, dims=dims, device=0)
    yield sc, field
    sc.close()


@pytest.mark.parametrize("el,az,radius,n", SUNS)
@pytest.mark.parametrize("extra", [0, "pool"])
def test_doom_frames_and_counters_equal_the_oracle(small, noise, el, az, radius, n, extra):
    import oracle
    import voxmap_amd as vx
    sc, field = small
    if extra == "pool" and n <= 1:
        pytest.skip("the pooled soft-shadow pass needs samples")
    o = oracle.Oracle(sc.read_field(), noise, exit=True)
    base = vx.FLAG_FULL_QUALITY | (vx.FLAG_SOFT_POOL if extra == "pool" else 0)
    got = {}
    for fl in (0, vx.FLAG_NO_DOOM):
        fr = vx.make_frame((48.0, 32.0, 36.0), (1.1, 0.0, 0.5), 96, 64, sun=_sun(el, az), flags=base | fl,
                           shadow_samples=n, sun_radius=radius)
        img, st = sc.render(fr, stats=True)
        ref, ost = o.render(fr.params, 96, 64)
        assert np.array_equal(img.view(np.uint32), ref.view(np.uint32)), (el, az, fl)
        a, b = st.as_dict(), ost.as_dict()
        assert a["shadow_fetches"] == b["shadow_fetches"], (el, az, fl, a["shadow_fetches"], b["shadow_fetches"])
        assert a["shadow_rays"] == b["shadow_rays"]
        got[fl] = (img, a["shadow_fetches"])
    assert np.array_equal(got[0][0].view(np.uint32), got[vx.FLAG_NO_DOOM][0].view(np.uint32))
    assert got[0][1] <= got[vx.FLAG_NO_DOOM][1]


@pytest.mark.parametrize("max_steps", [12, 20, 30, 44])
def test_doom_step_budgets(small, noise, max_steps):
    """Short march budgets (max_shadow_steps): hmax shrinks with MAX, a code read
    late in a march goes on from the cell's texel (read from the plain channel),
    and a budget too short for any h builds no table; frames and counters equal
    the oracle's, frames equal the no-doom frames."""
    import oracle
    import voxmap_amd as vx
    sc, _ = small
    o = oracle.Oracle(sc.read_field(), noise, exit=True)
    for el, az, radius, n in SUNS[:7]:
        got = []
        for fl in (0, vx.FLAG_NO_DOOM):
            fr = vx.make_frame((48.0, 32.0, 36.0), (1.1, 0.0, 0.5), 96, 64, sun=_sun(el, az),
                               flags=vx.FLAG_FULL_QUALITY | fl, shadow_samples=n, sun_radius=radius,
                               max_shadow_steps=max_steps)
            img, st = sc.render(fr, stats=True)
            ref, ost = o.render(fr.params, 96, 64)
            assert np.array_equal(img.view(np.uint32), ref.view(np.uint32)), (el, az, fl)
            assert st.as_dict()["shadow_fetches"] == ost.as_dict()["shadow_fetches"], (el, az, fl)
            got.append(img)
        assert np.array_equal(got[0].view(np.uint32), got[1].view(np.uint32))


def test_soft_brick_frames_read_no_doom_codes(small, noise):
    """VX_FLAG_SOFT_BRICK frames read a cone copy without the table (its LDS
    brick march has no doom rule): same frame as the default, counters equal
    the oracle's, which skips the table for that flag too."""
    import oracle
    import voxmap_amd as vx
    sc, _ = small
    o = oracle.Oracle(sc.read_field(), noise, exit=True)
    for el, az, radius, n in SUNS[5:]:
        imgs = []
        for fl in (vx.FLAG_SOFT_POOL | vx.FLAG_SOFT_BRICK, 0):
            fr = vx.make_frame((48.0, 32.0, 36.0), (1.1, 0.0, 0.5), 96, 64, sun=_sun(el, az),
                               flags=vx.FLAG_FULL_QUALITY | fl, shadow_samples=n, sun_radius=radius)
            img, st = sc.render(fr, stats=True)
            _, ost = o.render(fr.params, 96, 64)
            assert st.as_dict()["shadow_fetches"] == ost.as_dict()["shadow_fetches"], (el, az, fl)
            imgs.append(img)
        assert np.array_equal(imgs[0].view(np.uint32), imgs[1].view(np.uint32))


@pytest.mark.parametrize("cfg,scene,w,h", [("C5", "s_proc", 3840, 2160), ("C5", "s_glass", 3840, 2160),
                                           ("C5", "s_up3", 1920, 1080)])
def test_bench_workloads_identical_with_fewer_fetches(cfg, scene, w, h):
    """Full-size property: the doom frame equals the no-doom frame (itself
    oracle-pinned by the suites above and tests/test_exit_gpu.py) in RGBA32F,
    cameras K0-K2, and the table removes shadow fetches."""
    import voxmap_amd as vx
    from voxmap_amd import presets
    from voxmap_amd import scenes
    grid = presets.scene_grid(scene)
    Z, Y, X = grid.shape
    sc = vx.Scene(map_bytes=grid.tobytes(), map_format=vx.FORMAT_GRID, noise_path=scenes.NOISE_PATH,
                  dims=(X, Y, Z), device=0)            # the bench's scene (field built on the device)
    try:
        scale = 3.0 if scene == "s_up3" else 1.0
        samples = presets.CONFIGS[cfg].get("samples", 0)
        saved = 0
        for cam in ("K0", "K1", "K2"):
            res = {}
            for fl in (0, vx.FLAG_NO_DOOM):
                fr = presets.camera_frame(cam, w, h, scale=scale, flags=vx.FLAG_FULL_QUALITY | fl,
                                          shadow_samples=samples, sun_radius=0.03 if samples else 0.0)
                img, st = sc.render(fr, stats=True)
                res[fl] = (img, st.as_dict()["shadow_fetches"])
            assert np.array_equal(res[0][0].view(np.uint32), res[vx.FLAG_NO_DOOM][0].view(np.uint32)), cam
            assert res[0][1] <= res[vx.FLAG_NO_DOOM][1]
            saved += res[vx.FLAG_NO_DOOM][1] - res[0][1]
        assert saved > 0
    finally:
        sc.close()
