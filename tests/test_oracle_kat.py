"""Known-answer tests that pin the CPU oracle (the reference ships no tests or
golden images; SURVEY.md §4, §8c item list (1)-(4)).

- exp2: against the exact 2^x;
- march(): against an independent numpy-float32 transliteration of
  render.frag:75-142 (cell sequence end state, step count, fetches);
- a single block's shadow footprint against analytic ray/box geometry;
- an empty map: every sun-facing ground fragment is lit;
- the sky colour against a float64 closed form of render.frag:163-205;
- primary visibility against analytic ray/plane hits, glass and the
  no-boundary-face rule of the greedy mesh (ccol() clamps, sdf.cpp:302-303).
"""
import math

import numpy as np
import pytest

f32 = np.float32


@pytest.fixture(scope="module")
def O(built):
    import oracle
    return oracle


def test_exp2_known_values(O):
    for n in range(-120, 120, 7):
        assert O.exp2(float(n)) == 2.0 ** n
    xs = np.linspace(-30, 30, 2001)
    worst = max(abs(O.exp2(float(f32(x))) / 2.0 ** float(f32(x)) - 1) for x in xs)
    assert worst < 4e-7, worst
    assert O.exp2(-200.0) == 0.0 and math.isinf(O.exp2(200.0))


def _field(grid):
    import voxmap_amd as vx
    return vx.field_build(grid)


def march_py(field, cell, fract, r, max_steps):
    """numpy-float32 transliteration of march() (render.frag:75-142)."""
    Z, Y, X, _ = field.shape
    c = [int(v) for v in cell]
    f = [f32(v) for v in fract]
    r = [f32(v) for v in r]
    sgn = [f32(1) if v > 0 else (f32(-1) if v < 0 else f32(0)) for v in r]
    safe = f32(1)
    d = f32(1) if r[2] > 0 else f32(0)
    step, fetches = 0, 0
    while step < max_steps and safe != 0:
        t = []
        for i in range(3):
            x = f32(-f[i]) * sgn[i]
            dd = f32(x - np.floor(x)) + f32(1e-4)
            with np.errstate(divide="ignore"):
                t.append(f32(dd / f32(abs(r[i]))))
        m = [f32(1) if t[0] <= min(t[1], t[2]) else f32(0), f32(1) if t[1] <= min(t[2], t[0]) else f32(0),
             f32(1) if t[2] <= min(t[0], t[1]) else f32(0)]
        with np.errstate(invalid="ignore"):
            v = [f32(m[i] * t[i]) for i in range(3)]
            ln = f32(np.sqrt(f32(f32(f32(v[0] * v[0]) + f32(v[1] * v[1])) + f32(v[2] * v[2]))))
        for i in range(3):
            f[i] = f32(f[i] + f32(f32(r[i] * safe) * ln))
            fl = f32(np.floor(f[i]))
            c[i] += 0 if np.isnan(fl) else int(fl)   # ivec3(floor(NaN)) := 0
            f[i] = f32(f[i] - fl)
        if c[0] >= X or c[1] >= Y or c[2] >= Z or min(c) < 0:
            return max_steps, c, f, fetches
        tx = field[c[2], c[1], c[0]]
        fetches += 1
        safe = f32(tx[0]) if d == 1 else f32(tx[1])
        step += 1
    return step, c, f, fetches


def test_march_matches_float32_transliteration(O):
    from voxmap_amd import scenes
    g = scenes.small_proc(31, dims=(64, 40, 16), n_boxes=14, n_glass=2)
    field = _field(g)
    o = O.Oracle(field, np.zeros((4, 4, 4), np.uint8))
    rng = np.random.default_rng(0)
    dirs = [(0.7287353, 0.42073548, 0.5403023), (0.0, 0.0, 1.0), (1.0, 0.0, 0.0), (0.6, 0.6, 0.52915026),
            (-0.3, 0.5, 0.8124038), (0.5773503, -0.5773503, 0.5773503), (0.1, 0.2, -0.9746794)]
    n = 0
    for k in range(2000):
        if n >= 48:
            break
        z = int(rng.integers(1, 8))
        x, y = int(rng.integers(0, 64)), int(rng.integers(0, 40))
        if g[z, y, x]:
            continue
        r = dirs[n % len(dirs)] if n < 14 else tuple(rng.normal(size=3) * [1, 1, 0.3] + [0, 0, 0.5])
        r = tuple(float(f32(v)) for v in np.asarray(r) / np.linalg.norm(r))
        fr = (float(f32(rng.random())), float(f32(rng.random())), 0.0)
        m = o.march((x, y, z), fr, r, 32)
        step, c, f, fetches = march_py(field, (x, y, z), fr, r, 32)
        assert m.step == step and m.fetches == fetches, (k, m.step, step)
        if step < 32:
            assert list(m.cell) == c and all(f32(a) == b for a, b in zip(m.fract, f))
        n += 1
    assert n > 30


def test_single_block_shadow_footprint(O):
    """Ground fragments (top face, z = 1 plane) are shadowed exactly where the
    sun ray meets the block's box, away from the box silhouette."""
    from voxmap_amd import scenes
    g = scenes.single_block(dims=(64, 32, 16), at=(20, 12, 1), color=5)
    g[1:6, 12, 20] = 5                       # a 1x1x5 column
    field = _field(g)
    o = O.Oracle(field, np.zeros((4, 4, 4), np.uint8))
    s = np.array([0.6, 0.2, 0.77])
    s = s / np.linalg.norm(s)
    sun = tuple(float(f32(v)) for v in s)
    lo, hi = np.array([20.0, 12.0, 1.0]), np.array([21.0, 13.0, 6.0])
    shadowed = agree = 0
    for y in range(6, 16):
        for x in range(12, 24):
            for fx, fy in [(a, b) for a in (0.1, 0.3, 0.5, 0.7, 0.9) for b in (0.15, 0.5, 0.85)]:
                if g[1, y, x]:
                    continue
                P = np.array([x + fx, y + fy, 1.0])
                with np.errstate(divide="ignore"):
                    t0 = (lo - P) / s
                    t1 = (hi - P) / s
                tn, tf = np.max(np.minimum(t0, t1)), np.min(np.maximum(t0, t1))
                hit = tn < tf and tf > 0
                margin = tf - tn
                m = o.march((x, y, 1), (fx, fy, 0.0), sun, 32)
                lit = m.step == 32
                if abs(margin) < 0.1:
                    continue                    # grazing the silhouette
                assert lit == (not hit), (x, y, fx, fy, margin)
                agree += 1
                shadowed += hit
    assert shadowed >= 6 and agree > 200


def test_empty_map_every_sun_facing_fragment_lit(O):
    import voxmap_amd as vx
    g = np.zeros((16, 96, 128), np.uint8)
    g[0] = 2
    field = _field(g)
    noise = np.full((8, 8, 4), 128, np.uint8)
    o = O.Oracle(field, noise)
    fr = vx.make_frame((64.0, 48.0, 10.0), (1e-4, 0.0, -0.002), 64, 48)
    img, st = o.render(fr.params, 64, 48)
    assert st.block_px == 64 * 48 and st.shadow_rays == 64 * 48
    # every pixel sees the lit ground top: lightCol = shadeCol + litCol * sqrt(n.sun)
    assert np.ptp(img[..., 0]) < 0.02


def _sky_closed_form(ray, sun, t, cam_xy, noise_a):
    """float64 closed form of render.frag:148-205 for a constant-alpha noise texture."""
    ray = np.asarray(ray, float) / np.linalg.norm(ray)
    n = np.array([-1.0, 0, 0])
    refl = ray - 2 * np.dot(n, ray) * n
    sunCol = np.array([1.4, 1.0, 0.5])
    sf = max(0.0, float(np.dot(sun, ray))) - 1
    sf = 2 ** (4000 * sf) + 0.3 * 2 ** (8 * sf)
    scatter = 1 - math.sqrt(max(0.0, sun[2]))
    mix = lambda a, b, w: np.asarray(a) * (1 - w) + np.asarray(b) * w
    space = mix([0.2, 0.4, 0.7], [0.2, 0.3, 0.5], scatter)
    scat = mix([0.7, 0.9, 1.0], [1.0, 0.3, 0.2], scatter)
    atm = mix(scat, space, math.sqrt(max(0.0, refl[2])))
    sky = np.clip(sunCol * sf + atm, 0, 1)
    if noise_a is None:
        return sky
    fb = 1 - 2 * noise_a / 255.0
    rz = abs(ray[2])
    cloud = 2 ** (6 * (fb - 1))
    cloudCol = mix(sunCol, [0.8] * 3, math.sqrt(cloud))
    mpos = ray[0] / ray[1]
    mh = (1 - fb) / (math.exp(0.3 * mpos * mpos) * 6)
    mf = 2 - fb
    if mh > rz and ray[1] > 0 and rz > 0:
        return mix(sky, sky * np.array([0.7, 0.8, 0.7]), mf * rz)
    return mix(sky, cloudCol, cloud)


@pytest.mark.parametrize("clouds", [False, True])
def test_sky_colour_closed_form(O, clouds):
    import voxmap_amd as vx
    from oracle import OGbuf
    sun = vx.sun_from_hour(1.0)
    noise = np.full((8, 8, 4), 77, np.uint8)
    o = O.Oracle(np.zeros((2, 2, 2, 4), np.uint8), noise)
    fr = vx.make_frame((1.0, 1.0, 1.0), (0.5, 0.0, 0.1), 8, 8, sun=sun, flags=0 if clouds else vx.FLAG_NO_CLOUDS)
    g = OGbuf()
    g.id, g.normal_idx = 1, 1
    dirs = [(0.3, 0.9, 0.3), (0.7, 0.42, 0.54), (-0.2, 0.1, 0.97), (0.5, -0.8, 0.1), (0.9, 0.05, 0.02),
            (-0.6, 0.6, 0.5), (0.2, 0.3, -0.9), (0.72873, 0.42073, 0.54030)]
    for d in dirs:
        got = np.array(o.shade(fr.params, g, d)[:3])
        want = _sky_closed_form(d, np.array(sun, float), fr.params.time, None, 77 if clouds else None)
        assert np.allclose(got, want, rtol=2e-5, atol=2e-6), (d, got, want)


def test_primary_hits_top_face_analytically(O):
    import voxmap_amd as vx
    from voxmap_amd import scenes
    g = scenes.single_block(dims=(64, 32, 16), at=(20, 12, 1), color=5)
    field = _field(g)
    o = O.Oracle(field, np.zeros((4, 4, 4), np.uint8))
    fr = vx.make_frame((20.4, 12.7, 4.0), (0.08, 0.0, 0.2), 48, 48)
    p = fr.params
    cam = np.array(p.cam_cell, float) + np.array(p.cam_fract, float)
    hits = 0
    for px in range(0, 48):
        for py in range(0, 48):
            d = np.array(o.pixel_dir(p, 48, 48, px, py), float)
            n, gb, fetches, cap = o.primary(p, d)
            assert cap == 0 and n >= 1
            h = gb[0]
            t = (2.0 - cam[2]) / d[2]                  # plane z = 2: top of the block
            P = cam + t * d
            if 20 < P[0] < 21 and 12 < P[1] < 13 and min(P[0] - 20, 21 - P[0], P[1] - 12, 13 - P[1]) > 1e-3:
                assert (h.id, h.color, h.normal_idx) == (0, 5, 4)
                assert list(h.cell) == [20, 12, 2] and h.fract[2] == 0.0
                assert abs(h.cell[0] + h.fract[0] - P[0]) < 1e-4 and abs(h.cell[1] + h.fract[1] - P[1]) < 1e-4
                hits += 1
            else:
                t0 = (1.0 - cam[2]) / d[2]             # else the ground top at z = 1
                Q = cam + t0 * d
                if not (19.9 < Q[0] < 21.1 and 11.9 < Q[1] < 13.1):
                    assert (h.color, h.normal_idx, h.cell[2]) == (2, 4, 1)
    assert hits >= 20


def test_primary_glass_then_behind_and_boundary_rule(O):
    """sdf.cpp remaps air to B = pal_size = 22 (sdf.cpp:19,188,229-233) and
    meshes only colours < pal_size (:284): air is never a surface, the glass
    pane's far side is a back face (culled, render.js:88-91), so the wall
    behind the pane is what the glass blends over."""
    import voxmap_amd as vx
    g = np.zeros((8, 16, 32), np.uint8)
    g[0] = 2
    g[1:4, 8, 10:20] = 21          # a glass pane (y = 8)
    g[1:4, 12, 10:20] = 7          # a wall behind it (y = 12)
    g[1:6, 0:16, 31] = 9           # a wall on the grid's x = 31 edge
    field = _field(g)
    assert (field[g == 0][:, 2] == 22).all()          # map.bin air is B = pal_size
    o = O.Oracle(field, np.zeros((4, 4, 4), np.uint8))
    fr = vx.make_frame((15.0, 4.0, 2.0), (math.pi / 2, 0.0, 0.0), 16, 16)   # looking +y, level
    d = np.array([0.0, 1.0, 0.01])
    n, gb, _, cap = o.primary(fr.params, d)
    assert n == 2 and gb[0].id == 2 and gb[0].color == 21 and gb[0].normal_idx == 3   # -y face of the pane
    assert list(gb[0].cell)[1] == 8
    # behind the pane: the wall's -y face at y = 12 (glass -> air is no face)
    assert gb[1].color == 7 and gb[1].id == 0 and gb[1].normal_idx == 3 and gb[1].cell[1] == 12
    # entering the grid through its x = 31 edge straight into a block: no face there (ccol clamps);
    # leaving the block into air is its back face (culled) and air has none: sky
    fr2 = vx.make_frame((40.0, 5.5, 2.0), (math.pi / 2, 0.0, math.pi / 2), 16, 16)
    d2 = np.array([-1.0, 0.001, 0.002])
    n2, gb2, _, _ = o.primary(fr2.params, d2)
    assert n2 == 0
    # two panes: single blend layer, the second pane is skipped, the wall is behind
    g2 = g.copy()
    g2[1:4, 10, 10:20] = 21
    o2 = O.Oracle(_field(g2), np.zeros((4, 4, 4), np.uint8))
    n3, gb3, _, _ = o2.primary(fr.params, d)
    assert n3 == 2 and gb3[0].color == 21 and gb3[0].cell[1] == 8 and gb3[1].color == 7 and gb3[1].cell[1] == 12
    # glass directly against the wall: the wall's face toward the glass is the surface behind
    g3 = g.copy()
    g3[1:4, 9:12, 10:20] = 21
    o3 = O.Oracle(_field(g3), np.zeros((4, 4, 4), np.uint8))
    n4, gb4, _, _ = o3.primary(fr.params, d)
    assert n4 == 2 and gb4[1].color == 7 and gb4[1].cell[1] == 12


def test_air_encoding_b22_equals_b0_and_unmeshed_colours(O):
    """The same scene with air written as B = 22 (sdf.cpp) and as B = 0 (a
    pre-remap grid) renders identically, with identical work counters.  A
    block whose B is not a meshed index (>= pal_size, e.g. a black map colour
    that sdf.cpp remaps to pal_size) shows no face but still casts shadows
    (R = G = 0)."""
    import voxmap_amd as vx
    from voxmap_amd import scenes
    g = scenes.small_proc(23, dims=(64, 40, 16), n_boxes=12, n_glass=6)
    f22 = _field(g)
    f0 = f22.copy()
    f0[..., 2][g == 0] = 0
    noise = vx.noise_synth(0)
    fr = vx.make_frame((32.0, 20.0, 18.0), (1.1, 0.0, 0.6), 80, 60)
    a, sa = O.Oracle(f22, noise).render(fr.params, 80, 60)
    b, sb = O.Oracle(f0, noise).render(fr.params, 80, 60)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
    assert sa.as_dict() == sb.as_dict()
    # unmeshed block: invisible, but its R = G = 0 stops the sun march
    g4 = np.zeros((8, 16, 16), np.uint8)
    g4[0] = 2
    g4[3, 8, 8] = 5
    f4 = _field(g4)
    f4[3, 8, 8, 2] = 22
    o4 = O.Oracle(f4, noise)
    n, gb, _, _ = o4.primary(vx.make_frame((8.5, 8.5, 7.0), (1e-4, 0.0, 0.0), 8, 8).params, (0.0, 0.0, -1.0))
    assert n == 1 and gb[0].color == 2 and gb[0].cell[2] == 1        # straight through to the ground
    sun = np.array([0.1, 0.05, 0.99]) / np.linalg.norm([0.1, 0.05, 0.99])
    m = o4.march((8, 8, 1), (0.5, 0.5, 0.0), tuple(float(f32(v)) for v in sun), 16)
    assert m.step < 16                                                 # the march stops on the block


def test_field_octant_is_air_cube_ahead(O):
    """Octant cube size r: the cube [c, c + r*s] (s = the octant's direction signs)
    holds no non-air cell, r + 1 <= cap, and r is maximal: brute force over every
    cell and octant on a small random grid (cells outside the grid count as air)."""
    rng = np.random.default_rng(3)
    Z, Y, X, cap = 7, 9, 11, 5
    col = np.where(rng.random((Z, Y, X)) < 0.05, 7, 0).astype(np.uint8)
    field = np.zeros((Z, Y, X, 4), np.uint8)
    field[..., 2] = col
    solid = col != 0
    for oct in range(8):
        s = [-1 if oct & b else 1 for b in (1, 2, 4)]        # x, y, z signs
        got = O.field_octant(field, oct, cap)
        for z in range(Z):
            for y in range(Y):
                for x in range(X):
                    L = 0
                    while L < cap:                           # grow the cube while it stays air
                        xs = [x + s[0] * k for k in range(L + 1)]
                        ys = [y + s[1] * k for k in range(L + 1)]
                        zs = [z + s[2] * k for k in range(L + 1)]
                        xs = [v for v in xs if 0 <= v < X]
                        ys = [v for v in ys if 0 <= v < Y]
                        zs = [v for v in zs if 0 <= v < Z]
                        if solid[np.ix_(zs, ys, xs)].any():
                            break
                        L += 1
                    assert got[z, y, x] == max(L - 1, 0), (oct, x, y, z, got[z, y, x], L)
        assert got.max() <= cap - 1                   # 255 stays free for the out-of-grid sentinel
