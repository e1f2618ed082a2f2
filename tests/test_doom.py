"""The sun doom table (DESIGN.md §3 "Doom table") in the oracle, on the CPU.

vxo_field_doom is pinned against an independent numpy restatement of its
definition (window maxima by padding and shifting, the sun's x / y signs by
mirroring the grid), and the oracle's frames with the table equal its frames
without it (VX_FLAG_NO_DOOM), bit for bit, with fewer shadow fetches: the table
only ends marches early that end unlit anyway.  The kernel's table and march
are held to the same oracle by tests/test_doom_gpu.py."""
import math

import numpy as np
import pytest

NO_DOOM = 0x20000       # include/voxmap.h VX_FLAG_NO_DOOM (oracle/vxo.h VXO_FLAG_NO_DOOM)
Q, EPS, HCAP = 8, 1.0 / 64.0, 120


def _wmax(D, lo, hi, axis):
    """out[i] = max over k in [lo, hi] of D[i + k] along axis (outside: 255)."""
    n = D.shape[axis]
    pad_lo, pad_hi = max(0, -lo), max(0, hi)
    pw = [(0, 0), (0, 0)]
    pw[axis] = (pad_lo, pad_hi)
    P = np.pad(D, pw, constant_values=255)
    out = None
    for k in range(lo, hi + 1):
        sl = [slice(None), slice(None)]
        sl[axis] = slice(pad_lo + k, pad_lo + k + n)
        v = P[tuple(sl)]
        out = v.copy() if out is None else np.maximum(out, v)
    return out


def _doom_numpy(field, dirs, max_steps):
    """Depth recursion over Q x Q sub-cells per cell, top layer down, in the
    sun-aligned grid (x, y mirrored where the sun's component is negative);
    h up to the largest value the stop rule can use at landing 1; a doomed
    cell holds its crossing bound C(h)."""
    d = np.asarray(dirs, np.float32).reshape(-1, 3)
    hmax = 0
    ax = np.abs(d[:, 0].astype(np.float64) / d[:, 2].astype(np.float64))
    ay = np.abs(d[:, 1].astype(np.float64) / d[:, 2].astype(np.float64))
    xlo, xhi = math.floor(Q * (ax.min() - EPS)), math.ceil(Q * (ax.max() + EPS))
    ylo, yhi = math.floor(Q * (ay.min() - EPS)), math.ceil(Q * (ay.max() + EPS))
    sx, sy = (1 if d[0, 0] > 0 else -1), (1 if d[0, 1] > 0 else -1)
    cross = lambda h: h + (h * xhi) // Q + 1 + (h * yhi) // Q + 1       # boundary crossings to the block
    while hmax < HCAP and cross(hmax + 1) <= HCAP and 1 + 2 * cross(hmax + 1) < max_steps:
        hmax += 1
    solid = (field[..., 0] == 0) & (field[..., 1] == 0)
    if sx < 0:
        solid = solid[:, :, ::-1]
    if sy < 0:
        solid = solid[:, ::-1, :]
    Z, Y, X = solid.shape
    # the cells covering sub-cell g widened by 1/64 cell: floor((g -+ Q eps) / Q)
    gx, gy = np.arange(X * Q), np.arange(Y * Q)
    cx0, cx1 = np.floor((gx - EPS * Q) / Q).astype(int), np.floor((gx + 1 + EPS * Q) / Q).astype(int)
    cy0, cy1 = np.floor((gy - EPS * Q) / Q).astype(int), np.floor((gy + 1 + EPS * Q) / Q).astype(int)
    D1 = np.full((Y * Q, X * Q), 255, np.uint8)
    code = np.zeros((Z, Y, X), np.uint8)
    for z in range(Z - 1, -1, -1):
        m = _wmax(_wmax(D1, -1, Q + xhi, 1), -1, Q + yhi, 0)[::Q, ::Q]
        h = m.astype(np.int32) + 1
        cr = np.array([cross(int(v)) if v <= hmax else 0 for v in range(256)], np.int32)
        code[z] = np.where((m < 255) & (h <= hmax) & ~solid[z], cr[np.minimum(h, 255)], 0)
        s = solid[z]

        def cov(cy, cx):
            ok = ((cy >= 0) & (cy < Y))[:, None] & ((cx >= 0) & (cx < X))[None, :]
            return ok & s[np.clip(cy, 0, Y - 1)][:, np.clip(cx, 0, X - 1)]
        es = cov(cy0, cx0) & cov(cy0, cx1) & cov(cy1, cx0) & cov(cy1, cx1)
        w = _wmax(_wmax(D1, xlo, xhi, 1), ylo, yhi, 0)
        D1 = np.where(es, 0, np.where(w < 255, np.minimum(w.astype(np.int32) + 1, 254), 255)).astype(np.uint8)
    if sy < 0:
        code = code[:, ::-1, :]
    if sx < 0:
        code = code[:, :, ::-1]
    return np.ascontiguousarray(code), (sx, sy, xlo, xhi, ylo, yhi, hmax)


def _sun(el_deg, az_deg):
    el, az = math.radians(el_deg), math.radians(az_deg)
    return (math.cos(el) * math.cos(az), math.cos(el) * math.sin(az), math.sin(el))


# every sign pattern of (r_x, r_y) with r_z > 0, steep to low (slopes up to 4)
# (radius, samples): hard and soft shadows
SUNS = [(33, 30, 0.02, 4), (40, 120, 0.02, 4), (60, 210, 0.03, 8), (20, 300, 0.02, 2), (15, 45, 0.01, 4),
        (45, 160, 0.05, 8), (33, 30, 0.0, 1), (15, 45, 0.0, 1)]


@pytest.fixture(scope="module")
def field(built):
    import voxmap_amd as vx
    from voxmap_amd import scenes
    return vx.field_build(scenes.small_proc(31, dims=(96, 64, 40), n_boxes=30, n_glass=5))


@pytest.mark.parametrize("el,az,radius,n", SUNS)
@pytest.mark.parametrize("max_steps", [0, 200])
def test_field_doom_matches_numpy_restatement(field, el, az, radius, n, max_steps):
    import oracle
    d = oracle.sun_samples(_sun(el, az), radius, n)
    cone, _, kx, ky = oracle.exit_plan(d)
    assert cone
    maxs = max_steps or 2 * field.shape[0]            # render.frag:12 (2 Z), or a frame's own
    ref, plan = _doom_numpy(field, d, maxs)
    assert oracle.doom_plan(d, maxs) == plan
    got = oracle.field_doom(field, plan)
    assert got.shape == ref.shape
    assert np.array_equal(got, ref), int((got != ref).sum())
    assert int((got > 0).sum()) > 0                       # the scene has doomed cells


def test_doom_frames_identical_with_fewer_fetches(field, noise):
    import oracle
    import voxmap_amd as vx
    o = oracle.Oracle(field, noise, exit=True)
    saved = 0
    for el, az, radius, n in SUNS:
        a = vx.make_frame((48.0, 32.0, 36.0), (1.1, 0.0, 0.5), 96, 64, sun=_sun(el, az), flags=vx.FLAG_FULL_QUALITY,
                          shadow_samples=n, sun_radius=radius)
        b = vx.make_frame((48.0, 32.0, 36.0), (1.1, 0.0, 0.5), 96, 64, sun=_sun(el, az),
                          flags=vx.FLAG_FULL_QUALITY | NO_DOOM, shadow_samples=n, sun_radius=radius)
        ia, sa = o.render(a.params, 96, 64)
        ib, sb = o.render(b.params, 96, 64)
        assert np.array_equal(ia.view(np.uint32), ib.view(np.uint32)), (el, az)
        fa, fb = sa.as_dict()["shadow_fetches"], sb.as_dict()["shadow_fetches"]
        assert fa <= fb, (el, az)
        assert sa.as_dict()["shadow_rays"] == sb.as_dict()["shadow_rays"]
        saved += fb - fa
    assert saved > 0
    # short budgets: codes resolved late go on from the texel; no table when no h fits
    for maxs in (12, 20, 30):
        for el, az, radius, n in SUNS[:3]:
            fa = vx.make_frame((48.0, 32.0, 36.0), (1.1, 0.0, 0.5), 96, 64, sun=_sun(el, az),
                               flags=vx.FLAG_FULL_QUALITY, shadow_samples=n, sun_radius=radius, max_shadow_steps=maxs)
            fb = vx.make_frame((48.0, 32.0, 36.0), (1.1, 0.0, 0.5), 96, 64, sun=_sun(el, az),
                               flags=vx.FLAG_FULL_QUALITY | NO_DOOM, shadow_samples=n, sun_radius=radius,
                               max_shadow_steps=maxs)
            ia, sa = o.render(fa.params, 96, 64)
            ib, sb = o.render(fb.params, 96, 64)
            assert np.array_equal(ia.view(np.uint32), ib.view(np.uint32)), (maxs, el, az)
            assert sa.as_dict()["shadow_fetches"] <= sb.as_dict()["shadow_fetches"]
    # the hard shadow reads the table too: a one-sample frame saves fetches
    a = vx.make_frame((48.0, 32.0, 36.0), (1.1, 0.0, 0.5), 96, 64, sun=_sun(15, 45), flags=vx.FLAG_FULL_QUALITY)
    b = vx.make_frame((48.0, 32.0, 36.0), (1.1, 0.0, 0.5), 96, 64, sun=_sun(15, 45),
                      flags=vx.FLAG_FULL_QUALITY | NO_DOOM)
    assert o.render(a.params, 96, 64)[1].as_dict()["shadow_fetches"] < \
        o.render(b.params, 96, 64)[1].as_dict()["shadow_fetches"]
