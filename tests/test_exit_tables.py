"""The build's sun exit tables (DESIGN.md §3 "Sun exit tables"), on CPU.

The kernel's sun march reads a copy of the march channel in which every cell
from which the march cannot end unlit holds -1 (its "left the grid" mark), so
such a march stops there, lit, instead of stepping on to the grid edge or to
MAX_STEPS (render.frag:92-136, 234).  The oracle restates the tables
(oracle/vxo_field.c vxo_field_exit) and the per-frame choice (vxo_exit_plan);
here they are checked against brute-force definitions, and the soundness of
the exit -- no pixel changes -- over random suns, scenes and cameras.
"""
import math

import numpy as np
import pytest


def _field(seed, dims=(64, 40, 16), n_boxes=8, n_glass=2):
    import voxmap_amd as vx
    from voxmap_amd import scenes
    return vx.field_build(scenes.small_proc(seed, dims=dims, n_boxes=n_boxes, n_glass=n_glass))


def _brute(field, oct, kx, ky):
    """D by the layer recursion of the definition, one cell at a time."""
    Z, Y, X, _ = field.shape
    sx, sy, sz = (1 if oct & 1 else -1), (1 if oct & 2 else -1), (1 if oct & 4 else -1)
    T = field[..., 0] if sz > 0 else field[..., 1]
    D = np.zeros((Z, Y, X), np.uint8)
    zs = range(Z - 1, -1, -1) if sz > 0 else range(Z)
    for z in zs:
        zn = z + sz
        for y in range(Y):
            for x in range(X):
                ok = True
                ii = range(X) if kx < 0 else range(kx + 1)
                jj = range(Y) if ky < 0 else range(ky + 1)
                for j in jj:
                    yy = y + j * sy
                    if not 0 <= yy < Y:
                        break
                    for i in ii:
                        xx = x + i * sx
                        if not 0 <= xx < X:
                            break
                        nxt = True if not 0 <= zn < Z else bool(D[zn, yy, xx])
                        if T[z, yy, xx] == 0 or not nxt:
                            ok = False
                            break
                    if not ok:
                        break
                D[z, y, x] = ok
    return D


@pytest.mark.parametrize("oct", range(8))
def test_orthant_table_is_the_empty_orthant(built, oct):
    """Unbounded window: 1 iff no 0 texel of the octant's channel in the orthant ahead."""
    import oracle
    f = _field(3, dims=(48, 32, 16), n_boxes=5, n_glass=1)
    Z, Y, X, _ = f.shape
    T = f[..., 0] if oct & 4 else f[..., 1]
    e = oracle.field_exit(f, oct)
    for z in range(Z):
        for y in range(Y):
            for x in range(X):
                xs = slice(x, X) if oct & 1 else slice(0, x + 1)
                ys = slice(y, Y) if oct & 2 else slice(0, y + 1)
                zs = slice(z, Z) if oct & 4 else slice(0, z + 1)
                assert e[z, y, x] == (0 if (T[zs, ys, xs] == 0).any() else 1), (x, y, z)
    assert 0 < e.sum() < e.size if oct & 4 else e.sum() == 0   # ground at z = 0: no down-going exit


@pytest.mark.parametrize("oct,kx,ky", [(7, 2, 1), (4, 1, 3), (5, 0, 2), (6, 4, 4), (7, 5, 0)])
def test_cone_table_matches_recursion(built, oct, kx, ky):
    import oracle
    f = _field(9, dims=(48, 32, 16), n_boxes=6, n_glass=1)
    assert np.array_equal(oracle.field_exit(f, oct, kx, ky), _brute(f, oct, kx, ky))


def test_exit_plan_rules(built):
    import oracle
    import voxmap_amd as vx
    sun = vx.sun_from_hour(1.0)                         # (0.7288, 0.4208, 0.5403): slopes 1.349, 0.779
    assert oracle.exit_plan([sun]) == (True, [7], 2, 1)
    assert oracle.exit_plan([sun], allow_cone=False) == (False, [7], -1, -1)
    soft = oracle.sun_samples(sun, 0.03, 16)
    cone, octs, kx, ky = oracle.exit_plan(soft)
    assert cone and octs == [7] * 16 and (kx, ky) == (2, 1)
    low = [0.95, 0.2, 0.2]                              # slope 4.75 > 4: orthant tables
    assert oracle.exit_plan([low])[0] is False
    down = [0.6, 0.4, -0.69]                            # r_z < 0: orthant (G channel)
    assert oracle.exit_plan([down]) == (False, [3], -1, -1)
    tiny = [0.8, 1e-4, 0.6]                             # a component below 2^-10: literal march
    assert oracle.exit_plan([tiny]) == (False, [-1], -1, -1)
    mixed = [[0.5, 0.02, 0.866], [0.5, -0.02, 0.866]]   # two sign patterns: orthant each
    assert oracle.exit_plan(mixed) == (False, [7, 5], -1, -1)
    # the window bound: exactly representable slope 2 needs kx = ceil(2 + 1/64) = 3
    assert oracle.exit_plan([[0.8, 0.2, 0.4]])[2:] == (3, 1)


def _suns(n, seed):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        el = rng.uniform(math.radians(8), math.radians(88))
        az = rng.uniform(0, 2 * math.pi)
        out.append((math.cos(el) * math.cos(az), math.cos(el) * math.sin(az), math.sin(el)))
    return out


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_exit_tables_change_no_pixel(built, seed, noise):
    """Random suns (elevation 8..88 degrees, any azimuth: cone and orthant
    tables, every octant of the sky), hard and 16-sample soft shadows, two
    cameras: the oracle with the tables renders bit-identical frames with no
    more shadow fetches, and every other counter equal."""
    import oracle
    import voxmap_amd as vx
    f = _field(20 + seed, dims=(64, 40, 16), n_boxes=14, n_glass=3)
    lit = oracle.Oracle(f, noise)
    ext = oracle.Oracle(f, noise, exit=True)
    cams = [((32.0, 20.0, 20.0), (1.0, 0.0, 0.7)), ((10.0, 30.0, 9.0), (1.35, 0.0, -2.2))]
    saved = 0
    for k, sun in enumerate(_suns(8, seed)):
        sbj, rot = cams[k % 2]
        samples = 16 if k % 3 == 2 else 0
        fr = vx.make_frame(sbj, rot, 64, 40, sun=sun, flags=vx.FLAG_FULL_QUALITY if k % 2 else 0,
                           shadow_samples=samples, sun_radius=0.05 if samples else 0.0)
        a, sa = lit.render(fr.params, 64, 40)
        b, sb = ext.render(fr.params, 64, 40)
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), (k, sun)
        da, db = sa.as_dict(), sb.as_dict()
        for key in da:
            if key == "shadow_fetches":
                assert db[key] <= da[key]
            else:
                assert da[key] == db[key], key
        saved += da["shadow_fetches"] - db["shadow_fetches"]
    assert saved > 0
