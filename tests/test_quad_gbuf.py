"""The raster's G-buffer split and its glass draw order, on the CPU oracle
(VERDICT r03 items 1-2).

- vxo_face_quads (per face: its offset from the origin of the greedy quad that
  covers it) against the quad-list restatement of sdf.cpp:281-356
  (oracle/mesh_ref.py), including dims that are not multiples of CHUNK;
- vxo_face_order (the vertex.bin emission order of a face's quad) against the
  order mesh_ref emits the glass quads in;
- the quad-relative split (v_cellPos = quad origin, v_fractPos = hit - origin,
  render.vert:25-28) equals the unit-cell split bit for bit where every face is
  its own quad (offsets all 0), and is what the oracle renders by default;
- glass in draw order (render.js:82-91: LESS, depth writes, SRC_ALPHA) equals
  the single layer wherever a ray crosses at most one pane, differs only on
  pixels crossing two or more, and for a ray toward -x through two parallel
  panes blends both (the far pane's quad is drawn first), toward +x one.
"""
import numpy as np
import pytest


@pytest.fixture(scope="module")
def O(built):
    import oracle
    return oracle


def per_face_from_quads(grid, quads):
    """(Z, Y, X, 6) offsets from mesh_ref's quad list (later duplicates overwrite
    earlier ones with the same value)."""
    Z, Y, X = grid.shape
    ref = np.full((Z, Y, X, 6), 0xFFFF, np.int64)
    for q in quads:
        x, y, z = (int(v) for v in q[0:3])
        du, dv = q[3:6], q[6:9]
        n = int(q[10])
        d = n // 2
        u, v = (d + 1) % 3, (d + 2) % 3
        for l in range(int(dv[v])):
            for k in range(int(du[u])):
                c = [x, y, z]
                c[u] += k
                c[v] += l
                if n % 2 == 0:
                    c[d] -= 1          # normal 0: the face's cell is behind the plane
                if 0 <= c[0] < X and 0 <= c[1] < Y and 0 <= c[2] < Z:
                    ref[c[2], c[1], c[0], n] = k | (l << 8)
    return ref


@pytest.mark.parametrize("seed,dims", [(0, (64, 32, 16)), (1, (70, 40, 16)), (2, (48, 48, 12))])
def test_face_quads_match_mesher(O, seed, dims):
    from oracle import mesh_ref
    from voxmap_amd import scenes
    g = scenes.small_proc(seed, dims=dims, n_boxes=10, n_glass=4)
    f = O.field_build(g)
    q = O.face_quads(f)
    ref = per_face_from_quads(g, mesh_ref.greedy_mesh(g))
    assert (q != 0xFFFF).sum() > 1000
    assert np.array_equal(q.astype(np.int64), ref)


def test_face_order_is_emission_order(O):
    import ctypes as C
    from oracle import mesh_ref
    from voxmap_amd import scenes
    g = scenes.s_glass(3, dims=(96, 64, 16), n_houses=6, n_facades=3)
    Z, Y, X = g.shape
    f = O.field_build(g)
    q = O.face_quads(f)
    quads = mesh_ref.greedy_mesh(g)
    glass = quads[quads[:, 9] == 21]
    assert len(glass) > 20
    last, seen = -1, {}
    for qd in glass:
        n = int(qd[10])
        d = n // 2
        cell = [int(v) for v in qd[0:3]]
        if n % 2 == 0:
            cell[d] -= 1
        off = int(q[cell[2], cell[1], cell[0], n])
        assert off == 0                                   # the quad's own origin face
        key = O.lib().vxo_face_order((C.c_int * 3)(*cell), n, off, X, Y, Z, 0)
        face = (tuple(cell), n)
        if face in seen:                                  # a chunk-plane face emitted again
            assert seen[face] == key and key < last
            continue
        assert key > last
        seen[face] = key
        last = key


def test_quad_split_equals_unit_split_for_unit_quads(O, noise):
    """A checkerboard of colours makes every face its own 1x1 quad: offsets 0,
    so both splits round the same point the same way."""
    import voxmap_amd as vx
    X, Y, Z = 40, 32, 12
    g = np.zeros((Z, Y, X), np.uint8)
    zz, yy, xx = np.indices((Z, Y, X))
    g[0] = 2 + ((xx[0] + yy[0]) % 2) * 9
    pil = ((xx % 6 < 3) & (yy % 5 < 2) & (zz < 7) & (zz > 0))
    g[pil] = (1 + (xx + yy + zz) % 2 * 4)[pil]
    f = O.field_build(g)
    q = O.face_quads(f)
    assert np.all((q == 0xFFFF) | (q == 0))
    fr = vx.make_frame((X / 2, Y / 2, 10.0), (1.1, 0.0, 0.6), 96, 64, flags=vx.FLAG_FULL_QUALITY)
    a, sa = O.Oracle(f, noise, quad=False).render(fr.params, 96, 64)
    b, sb = O.Oracle(f, noise, quad=q).render(fr.params, 96, 64)
    assert sa.block_px > 1000
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


def test_quad_split_moves_fragments_onto_quad_origins(O):
    """The primary record's v_cellPos is the quad origin and v_cellPos +
    v_fractPos the same point as the unit cell's (to rounding)."""
    import voxmap_amd as vx
    X, Y, Z = 64, 40, 12
    g = np.zeros((Z, Y, X), np.uint8)
    g[0] = 2
    g[1:8, 10:30, 20:50] = 7                             # one box: big merged faces
    f = O.field_build(g)
    q = O.face_quads(f)
    A, B = O.Oracle(f, np.zeros((16, 16, 4), np.uint8), quad=False), O.Oracle(f, np.zeros((16, 16, 4), np.uint8), quad=q)
    fr = vx.make_frame((X / 2, Y / 2, 10.0), (1.1, 0.0, 0.6), 64, 48)
    moved = 0
    for py in range(0, 48, 5):
        for px in range(0, 64, 5):
            d = A.pixel_dir(fr.params, 64, 48, px, py)
            na, ga, _, _ = A.primary(fr.params, d)
            nb, gb, _, _ = B.primary(fr.params, d)
            assert na == nb
            for k in range(na):
                ax = ga[k].normal_idx // 2
                assert ga[k].cell[ax] == gb[k].cell[ax] and gb[k].fract[ax] == 0.0
                for i in range(3):
                    if i == ax:
                        continue
                    off = ga[k].cell[i] - gb[k].cell[i]
                    assert 0 <= off < Z
                    moved += off > 0
                    assert abs((gb[k].cell[i] + gb[k].fract[i]) - (ga[k].cell[i] + ga[k].fract[i])) < 1e-4
    assert moved > 50


def _two_panes():
    X, Y, Z = 48, 24, 12
    g = np.zeros((Z, Y, X), np.uint8)
    g[0] = 2
    g[1:10, 2:22, 12] = 21          # pane at x = 12
    g[1:10, 2:22, 20] = 21          # pane at x = 20
    g[1:10, 2:22, 2] = 9            # wall at x = 2
    g[1:10, 2:22, 30] = 9           # wall at x = 30
    return g


@pytest.mark.parametrize("yaw,both", [(-np.pi / 2, False), (np.pi / 2, True)])
def test_glass_order_two_panes(O, noise, yaw, both):
    """Looking along the panes' normal: from x = 25.3 toward -x the ray meets
    the pane at 20, the pane at 12, then the wall at 2 (the far pane's quad is
    drawn first: both blend); from x = 6.3 toward +x the pane at 12, the pane
    at 20, then the wall at 30 (the near pane first: the far one fails LESS)."""
    import voxmap_amd as vx
    g = _two_panes()
    f = O.field_build(g)
    Ob = O.Oracle(f, noise, quad=O.face_quads(f))
    # orbit camera (map.js:373-380): position = sbj + Rz(yaw) Rx(rx) (0, 0, sbj.z)
    x = 25.3 - 5.4 if both else 6.3 + 5.4
    fr = vx.make_frame((x, 12.2, 5.4), (1.5707, 0.0, yaw), 32, 32, flags=vx.FLAG_GLASS_SINGLE)
    fo = vx.make_frame((x, 12.2, 5.4), (1.5707, 0.0, yaw), 32, 32)
    a, _ = Ob.render(fr.params, 32, 32)
    b, _ = Ob.render(fo.params, 32, 32)
    n = Ob.glass_layers(fr.params, 32, 32)
    assert (n >= 2).sum() > 100
    diff = np.any(a.view(np.uint32) != b.view(np.uint32), axis=2)
    assert not np.any(diff & (n < 2))
    if both:
        assert diff[n >= 2].mean() > 0.9
    else:
        assert not diff.any()


def test_glass_order_changes_only_stacked_pixels(O, noise):
    import voxmap_amd as vx
    from voxmap_amd import scenes
    g = scenes.s_glass(2, dims=(96, 64, 16), n_houses=16, n_facades=4)
    f = O.field_build(g)
    Ob = O.Oracle(f, noise, exit=True, quad=O.face_quads(f))
    tot = 0
    for rot in ((1.1, 0.0, 0.6), (1.2, 0.0, 2.6), (1.3, 0.0, -2.2)):
        fr = vx.make_frame((48.0, 32.0, 20.0), rot, 128, 96, flags=vx.FLAG_FULL_QUALITY | vx.FLAG_GLASS_SINGLE)
        fo = vx.make_frame((48.0, 32.0, 20.0), rot, 128, 96, flags=vx.FLAG_FULL_QUALITY)
        a, sa = Ob.render(fr.params, 128, 96)
        b, sb = Ob.render(fo.params, 128, 96)
        n = Ob.glass_layers(fr.params, 128, 96)
        diff = np.any(a.view(np.uint32) != b.view(np.uint32), axis=2)
        assert not np.any(diff & (n < 2))
        assert sa.glass_px == sb.glass_px
        tot += int(diff.sum())
    assert tot > 20


def _many_panes(n_panes):
    """n_panes glass panes, 2 cells apart, between a wall at x = 2 and a camera
    at x ~ 45 looking toward -x: the far panes' quads are drawn first (lower
    chunk, lower slice), so every pane blends (render.js:82-91)."""
    X, Y, Z = 64, 24, 12
    g = np.zeros((Z, Y, X), np.uint8)
    g[0] = 2
    g[1:10, 2:22, 2] = 9
    for k in range(n_panes):
        g[1:10, 2:22, 38 - 3 * k] = 21     # nearest at x = 38, then 35, 32, ...
    return g


def test_glass_order_blends_more_than_eight_panes(O, noise):
    """Every pane a ray crosses takes part (no layer cap): with 10
    panes the two farthest still change the pixels that see them."""
    import voxmap_amd as vx
    fr = vx.make_frame((45.0 - 5.4, 12.2, 5.4), (1.5707, 0.0, np.pi / 2), 32, 32)
    imgs, layers = [], None
    for n in (10, 8):
        f = O.field_build(_many_panes(n))
        Ob = O.Oracle(f, noise, quad=O.face_quads(f))
        img, st = Ob.render(fr.params, 32, 32)
        imgs.append(img)
        if n == 10:
            layers = Ob.glass_layers(fr.params, 32, 32)
    assert (layers >= 9).sum() > 100, np.bincount(layers.ravel())
    diff = np.any(imgs[0].view(np.uint32) != imgs[1].view(np.uint32), axis=2)
    assert diff[layers >= 9].mean() > 0.9
