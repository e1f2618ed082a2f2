"""primary visibility vs the reference's own geometry.

The reference rasterises the greedy quad mesh of src/gen/sdf.cpp:281-356
(back-face culled, glass blended last, render.js:82-91; air remapped to
pal_size and never meshed); the build traverses the field instead.  oracle/mesh_ref.py restates the mesher and casts the same
fp32 camera rays against its quads in float64.  Every pixel whose hit is not
within 1e-3 of a quad border (where the raster's edge rules and the
traversal's x<y<z tie rule may legitimately differ) must show the same face:
colour, normal index and hit point (cell + fract, within 1e-3), for the glass
layer and the opaque layer behind it.
"""
import math

import numpy as np
import pytest

CASES = [
    # seed, dims, sbj, rot, n_glass
    (5, (64, 32, 16), (32.0, 16.0, 18.0), (1.1, 0.0, 0.6), 4),                 # oblique, K1-like
    (7, (64, 32, 16), (32.0, 16.0, 40.0), (1e-4, 0.0, -0.002), 4),             # top-down, K0-like
    (11, (64, 32, 16), (-6.0, 16.0, 9.0), (1.45, 0.0, -math.pi / 2), 10),      # grazing from outside, glass
    (13, (64, 32, 16), (32.0, 16.0, 6.0), (1.3, 0.0, 2.4), 4),                 # camera inside the grid
]
W, H = 96, 64


def _setup(case):
    import oracle
    import voxmap_amd as vx
    from oracle import mesh_ref
    from voxmap_amd import scenes
    seed, dims, sbj, rot, ng = case
    grid = scenes.small_proc(seed, dims=dims, n_boxes=12, n_glass=ng)
    field = vx.field_build(grid)
    noise = vx.noise_synth(0)
    fr = vx.make_frame(sbj, rot, W, H)
    O = oracle.Oracle(field, noise)
    p = fr.params
    dirs = np.array([O.pixel_dir(p, W, H, x, y) for y in range(H) for x in range(W)], np.float32)
    origin = np.array([p.cam_cell[i] + np.float64(p.cam_fract[i]) for i in range(3)])
    quads = mesh_ref.greedy_mesh(grid)
    hits = mesh_ref.cast(quads, origin, dirs.astype(np.float64))
    return grid, field, noise, fr, O, dirs, quads, hits


def test_mesher_faces_are_the_colour_changes(built):
    """Quad area per (colour, normal) == the number of unit faces between a
    cell of that (non-air) colour and a grid-adjacent cell of another colour,
    facing out of the coloured cell (boundary: none).  Air is remapped to
    pal_size (sdf.cpp:229-233) and never meshed (sdf.cpp:284): no quad has
    colour 0 or 22.
    Faces on interior chunk planes (multiples of CHUNK = Z) come out twice: the
    reference's slice p[d] = -1 of a chunk repeats the last slice of the chunk
    before it (sdf.cpp:299, a harmless quirk: identical coplanar quads)."""
    from oracle import mesh_ref
    from voxmap_amd import scenes
    grid = scenes.small_proc(5, dims=(64, 32, 16), n_boxes=12, n_glass=4)
    quads = mesh_ref.greedy_mesh(grid)
    col = np.transpose(grid, (2, 1, 0))                      # [x][y][z]
    CH = grid.shape[0]
    for d in range(3):
        a = np.take(col, np.arange(col.shape[d] - 1), axis=d)
        b = np.take(col, np.arange(1, col.shape[d]), axis=d)
        plane = np.arange(1, col.shape[d])                   # face between i and i+1 lies on plane i+1
        wshape = [1, 1, 1]
        wshape[d] = -1
        weight = np.where(plane % CH == 0, 2, 1).reshape(wshape)
        for c in np.unique(col):
            if c == 0:
                continue
            want_pos = int(np.sum(((a == c) & (b != c)) * weight))   # normal 2d: cell c on the low side
            want_neg = int(np.sum(((a != c) & (b == c)) * weight))   # normal 2d+1: cell c on the high side
            for nrm, want in ((0, want_pos), (1, want_neg)):
                sel = (quads[:, 9] == c) & (quads[:, 10] == 2 * d + nrm)
                area = int(np.sum(np.abs(quads[sel, 3:6]).sum(1) * np.abs(quads[sel, 6:9]).sum(1)))
                assert area == want, (d, int(c), nrm, area, want)
    # the reference's clamped ccol() leaves the grid boundary without faces
    assert not np.isin(quads[:, 9], (0, 22)).any()
    X = grid.shape[2]
    on_x_boundary = (quads[:, 10] // 2 == 0) & ((quads[:, 0] == 0) | (quads[:, 0] == X))
    assert not on_x_boundary.any()


@pytest.mark.parametrize("case", CASES, ids=["oblique", "top", "grazing_glass", "inside"])
def test_oracle_primary_matches_greedy_mesh(built, case):
    _, _, _, fr, O, dirs, quads, M = _setup(case)
    p = fr.params
    compared = glass_seen = 0
    bad = []
    for k, d in enumerate(dirs):
        if min(M["edge_opaque"][k], M["edge_glass"][k]) < 1e-3:
            continue
        n, gb, _, _ = O.primary(p, tuple(float(v) for v in d))
        recs = [gb[i] for i in range(n)]
        glass = recs[0] if n >= 1 and recs[0].id == 2 else None
        opaque = (recs[1] if n == 2 else None) if glass is not None else (recs[0] if n == 1 else None)
        for rec, qi, pt in ((glass, M["glass_q"][k], M["point_glass"][k]),
                            (opaque, M["opaque_q"][k], M["point_opaque"][k])):
            if rec is None or qi < 0:
                ok = rec is None and qi < 0
            else:
                q = quads[qi]
                ours = np.array([rec.cell[i] + np.float64(rec.fract[i]) for i in range(3)])
                # the record's v_cellPos is the quad's origin (render.vert:25: the
                # vert() records carry it, sdf.cpp:94-102) and v_cellPos + v_fractPos
                # the hit point
                ok = (rec.color == q[9] and rec.normal_idx == q[10]
                      and all(int(rec.cell[i]) == int(q[i]) for i in range(3))
                      and np.max(np.abs(ours - pt)) < 1e-3 * max(1.0, float(np.max(np.abs(pt)))))
            if not ok and len(bad) < 5:
                bad.append((k, n, int(qi)))
        compared += 1
        glass_seen += glass is not None
    assert not bad, bad
    assert compared >= 0.99 * len(dirs)
    if case[0] == 11:
        assert glass_seen > 50, glass_seen
        # glass over an opaque face behind it (the old air-face bug showed black there)
        assert np.sum((M["glass_q"] >= 0) & (M["opaque_q"] >= 0)) > 20


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES, ids=["oblique", "top", "grazing_glass", "inside"])
def test_hip_primary_only_matches_greedy_mesh(built, case):
    """libvoxmap_hip.so in PRIMARY_ONLY mode (palette colour of the first
    surface, BASELINE C1) against the nearest front face of the mesh."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU visible")
    import voxmap_amd as vx
    grid, field, noise, fr, _, dirs, quads, M = _setup(case)
    Z, Y, X = grid.shape
    fr.params.flags = vx.FLAG_PRIMARY_ONLY
    with vx.Scene(map_bytes=field.tobytes(), map_format=vx.FORMAT_BIN, noise_bytes=noise.tobytes(),
                  noise_format=vx.FORMAT_BIN, dims=(X, Y, Z), device=0) as sc:
        img, _ = sc.render(fr)
    img = img.reshape(-1, 4)
    from oracle import vxo_palette
    ok = np.minimum(M["edge_opaque"], M["edge_glass"]) >= 1e-3
    first = np.where(M["glass_q"] >= 0, M["glass_q"], M["opaque_q"])
    colour = np.where(first >= 0, quads[np.maximum(first, 0), 9], 0)
    want = vxo_palette()[colour]
    assert np.array_equal(img[ok, :3], want[ok]), int(np.sum(np.any(img[ok, :3] != want[ok], axis=1)))
    assert ok.mean() > 0.99


def test_glass_layer_count_matches_the_mesh(built):
    """The single-layer glass diagnostic (oracle.Oracle.glass_layers)
    against the restated mesher: two glass panes in front of a wall, seen from
    outside the grid.  Every non-edge pixel crosses as many front-facing glass
    quads of the greedy mesh (mesh_ref.cast n_glass) as the walk counts, and the
    pixels through both panes count 2 -- the pixels where the reference's
    draw-order blend and the build's one-layer blend can differ."""
    import oracle
    import voxmap_amd as vx
    from oracle import mesh_ref
    Z, Y, X = 16, 24, 48
    grid = np.zeros((Z, Y, X), np.uint8)
    grid[0] = 3                                   # ground
    grid[1:12, 4:20, 40:42] = 7                   # wall
    grid[1:12, 4:20, 20] = 21                     # glass pane 1 (x plane 20..21: not a chunk plane)
    grid[2:10, 6:18, 27] = 21                     # glass pane 2
    field = vx.field_build(grid)
    O = oracle.Oracle(field, np.zeros((16, 16, 4), np.uint8))
    w, h = 64, 48
    fr = vx.make_frame((-4.0, 12.0, 6.0), (math.pi / 2, 0.0, -math.pi / 2), w, h)
    p = fr.params
    n = O.glass_layers(p, w, h).ravel()
    dirs = np.array([O.pixel_dir(p, w, h, x, y) for y in range(h) for x in range(w)], np.float64)
    origin = np.array([p.cam_cell[i] + np.float64(p.cam_fract[i]) for i in range(3)])
    quads = mesh_ref.greedy_mesh(grid)
    M = mesh_ref.cast(quads, origin, dirs)
    ok = np.minimum(M["edge_opaque"], M["edge_glass"]) >= 1e-3
    assert ok.mean() > 0.9
    assert np.array_equal(n[ok], M["n_glass"][ok]), int(np.sum(n[ok] != M["n_glass"][ok]))
    assert np.sum(n == 2) > 100 and np.sum(n == 1) > 50
