"""Greedy-mesh cross-check of primary visibility — TEST INFRASTRUCTURE ONLY.

SURVEY §8 f-4.  The reference never ray-marches primary rays: it rasterises
the greedy quad mesh of src/gen/sdf.cpp:281-356 (vertex.bin) with depth test,
back-face culling and glass drawn last with alpha blending (render.js:82-91).
The build replaces that raster by a traversal of the field
(oracle/vxo_render.c walk(), vx_kernels.hip primary()).  This module restates
the mesher and intersects the camera rays with its quads, giving an
independent answer to "which face does this pixel show" to check the
traversal against.

Restated (read as text, not copied):
  * ccol(x, y, z): palette index with clamped coordinates (sdf.cpp:44-51), so
    the grid boundary has no faces;
  * cells hold map.bin's B: the remapped palette index, with AIR written as
    pal_size (sdf.cpp:19,188,229-233: pal[] is zero-initialised and scanned
    from 1, so air finds pal[pal_size] = 0);
  * for every colour c < pal_size (sdf.cpp:284: colour 0 never occurs after
    the remap and air = pal_size is never meshed), every chunk of
    CHUNK = Z cells per axis (voxmap.h:9, :62-67), every axis d and normal
    0/1, slices p[d] = -1 .. CHUNK-1 (sdf.cpp:299-311): mask = (normal 0:
    cell of colour c, cell ahead not) or (normal 1: cell not c, cell ahead c);
    the quad sits on plane p[d] + 1;
  * greedy merge in the (u, v) = ((d+1)%3, (d+2)%3) mask, width along u first,
    then height along v (sdf.cpp:313-351); quad (origin, du, dv, colour,
    normal index 2d + normal, id = 2 for glass = pal_size - 1 else 0);
  * normal index n faces +d for n even, -d for n odd (render.vert:14-17); the
    GL back-face cull keeps a face only for rays travelling against its normal;
  * quirk kept: slice p[d] = -1 of a chunk repeats the last slice of the chunk
    before it, so faces on interior chunk planes are emitted twice (identical
    coplanar quads; harmless for the raster and for the cast below).

Ray casting is float64 and reports, per ray, the nearest front-facing opaque
(non-glass) face, the nearest front-facing glass face in front of it, the
number of glass faces in front of it (the reference blends every one of them,
order-dependently; the build defines one layer) and the distance from the hit
point to the nearest quad edge (where raster edge rules and the traversal's
tie rules may legitimately pick different quads).
"""
from __future__ import annotations

import numpy as np

GLASS = 21  # pal_size - 1 (sdf.cpp:225, :337)


def remap_air(grid_zyx: np.ndarray, pal_size: int = 22) -> np.ndarray:
    """Palette grid (0 = air) -> map.bin's B channel: air becomes pal_size (sdf.cpp:229-233)."""
    g = np.asarray(grid_zyx)
    return np.where(g == 0, pal_size, g).astype(g.dtype)


def greedy_mesh(grid_zyx: np.ndarray, pal_size: int = 22) -> np.ndarray:
    """Quads of sdf.cpp:281-356 for a (Z, Y, X) palette grid (0 = air, remapped
    to pal_size first, as sdf.cpp does before meshing).

    Returns an int32 array (n, 12): x, y, z, du(3), dv(3), colour, normal, id.
    """
    g = remap_air(grid_zyx, pal_size)
    Z, Y, X = g.shape
    col = np.ascontiguousarray(np.transpose(g, (2, 1, 0)))   # col[x][y][z] as the reference indexes
    dims = (X, Y, Z)
    CH = Z                                                    # voxmap.h:9 CHUNK = Z
    quads = []
    for color in range(pal_size):
        is_c = col == color
        if not is_c.any():         # colour 0 (and unused colours): no quads
            continue
        for cx in range(0, X, CH):
            for cy in range(0, Y, CH):
                for cz in range(0, Z, CH):
                    base = (cx, cy, cz)
                    for d in range(3):
                        u, v = (d + 1) % 3, (d + 2) % 3
                        for normal in range(2):
                            for pd in range(-1, CH):
                                # mask over (p[v], p[u]) at slice p[d] = pd
                                iu = np.arange(CH)
                                iv = np.arange(CH)
                                P = [None, None, None]
                                P[d] = np.full((CH, CH), pd)
                                P[u] = np.broadcast_to(iu[None, :], (CH, CH))
                                P[v] = np.broadcast_to(iv[:, None], (CH, CH))
                                cur = [np.clip(base[k] + P[k], 0, dims[k] - 1) for k in range(3)]
                                ahd = [np.clip(base[k] + P[k] + (1 if k == d else 0), 0, dims[k] - 1)
                                       for k in range(3)]
                                block = is_c[cur[0], cur[1], cur[2]]
                                ahead = is_c[ahd[0], ahd[1], ahd[2]]
                                mask = (block & ~ahead) if normal == 0 else (~block & ahead)
                                if not mask.any():
                                    continue
                                mask = mask.copy()
                                plane = pd + 1                       # p[d]++ (sdf.cpp:311)
                                for j in range(CH):
                                    i = 0
                                    while i < CH:
                                        if not mask[j, i]:
                                            i += 1
                                            continue
                                        w = 1
                                        while i + w < CH and mask[j, i + w]:
                                            w += 1
                                        h = 1
                                        while j + h < CH and mask[j + h, i:i + w].all():
                                            h += 1
                                        p = [0, 0, 0]
                                        p[d] = plane
                                        p[u] = i
                                        p[v] = j
                                        du = [0, 0, 0]
                                        dv = [0, 0, 0]
                                        du[u] = w
                                        dv[v] = h
                                        cid = 2 if color == pal_size - 1 else 0
                                        quads.append([base[0] + p[0], base[1] + p[1], base[2] + p[2],
                                                      *du, *dv, color, d * 2 + normal, cid])
                                        mask[j:j + h, i:i + w] = False
                                        i += w
    return np.asarray(quads, dtype=np.int32).reshape(-1, 12)


def cast(quads: np.ndarray, origin, dirs: np.ndarray):
    """Intersect rays origin + t*dir (t > 0) with the front faces of ``quads``.

    dirs: (n, 3).  Returns a dict of per-ray arrays:
      opaque_q / glass_q: quad index of the nearest front-facing non-glass /
        glass face (glass only if in front of the opaque one), -1 if none;
      t_opaque / t_glass, point_opaque / point_glass (n, 3);
      n_glass: front-facing glass faces in front of the opaque hit;
      edge_opaque / edge_glass: distance of the hit point to its quad's border.
    """
    o = np.asarray(origin, np.float64)
    D = np.asarray(dirs, np.float64)
    n = D.shape[0]
    q = quads.astype(np.float64)
    org = q[:, 0:3]
    du, dv = q[:, 3:6], q[:, 6:9]
    nidx = quads[:, 10]
    ax = nidx // 2
    sgn = np.where(nidx % 2 == 0, 1.0, -1.0)                  # normal direction along ax
    glass = quads[:, 11] == 2
    out = {k: np.full(n, -1, np.int64) for k in ("opaque_q", "glass_q")}
    out.update({k: np.full(n, np.inf) for k in ("t_opaque", "t_glass", "edge_opaque", "edge_glass")})
    out["n_glass"] = np.zeros(n, np.int64)
    out["point_opaque"] = np.full((n, 3), np.nan)
    out["point_glass"] = np.full((n, 3), np.nan)
    lo = org + np.minimum(du, 0) + np.minimum(dv, 0)
    hi = org + np.maximum(du, 0) + np.maximum(dv, 0)
    chunk = max(1, 2_000_000 // max(1, len(quads)))
    for s in range(0, n, chunk):
        d = D[s:s + chunk]                                    # (m, 3)
        dax = d[:, ax]                                        # (m, Q)
        front = dax * sgn[None, :] < 0                        # travelling against the normal
        with np.errstate(divide="ignore", invalid="ignore"):
            plane = org[np.arange(len(quads)), ax]            # (Q,)
            t = (plane[None, :] - o[ax][None, :]) / dax
        t = np.where(front & (t > 0), t, np.inf)
        pts = o[None, None, :] + t[..., None] * d[:, None, :]  # (m, Q, 3)
        with np.errstate(invalid="ignore"):
            inside = np.all((pts >= lo[None] - 1e-9) & (pts <= hi[None] + 1e-9), axis=2)
        t = np.where(inside, t, np.inf)
        t_op = np.where(glass[None, :], np.inf, t)
        iop = np.argmin(t_op, axis=1)
        top = t_op[np.arange(len(d)), iop]
        t_gl = np.where(glass[None, :] & (t < top[:, None]), t, np.inf)
        igl = np.argmin(t_gl, axis=1)
        tgl = t_gl[np.arange(len(d)), igl]
        ng = np.sum(np.isfinite(t_gl), axis=1)
        rows = np.arange(len(d))
        for key_q, key_t, key_p, key_e, idx, tv in (("opaque_q", "t_opaque", "point_opaque", "edge_opaque", iop, top),
                                                    ("glass_q", "t_glass", "point_glass", "edge_glass", igl, tgl)):
            ok = np.isfinite(tv)
            out[key_q][s:s + chunk] = np.where(ok, idx, -1)
            out[key_t][s:s + chunk] = tv
            p = pts[rows, idx]
            out[key_p][s:s + chunk] = np.where(ok[:, None], p, np.nan)
            # distance to the quad border along the two in-plane axes
            pl, ph = lo[idx], hi[idx]
            e = np.minimum(p - pl, ph - p)
            e[rows, ax[idx]] = np.inf
            out[key_e][s:s + chunk] = np.where(ok, e.min(axis=1), np.inf)
        out["n_glass"][s:s + chunk] = ng
    return out


# ---- 2D mode mesh (sdf.cpp:362-401) and the vertex record layout ------------------
# The plaintext res/vertex2d.bin.gz is the one reference OUTPUT of the mesher that
# ships unencrypted.  Regenerating it byte for byte from the footprint it encodes
# pins the greedy merge order, the quad/triangle/record layout and the rule that
# air (c2d = pal_size after the remap, sdf.cpp:235-239) is never meshed.

REC2D = np.dtype([("p", "<i2", 3), ("d", "<i2", 3), ("c", "u1"), ("n", "u1"), ("id", "u1"), ("pad", "u1")])


def decode_vertex2d(raw: bytes, dims=(1024, 256), pal_size: int = 22) -> np.ndarray:
    """c2d[x][y] (X, Y) from vertex2d.bin bytes: each 6-vertex quad covers
    [x, x + w) x [y, y + h) with its colour; cells no quad covers are air
    (pal_size after the remap, sdf.cpp:235-239)."""
    rec = np.frombuffer(raw, REC2D)
    assert len(rec) % 6 == 0
    X, Y = dims
    c2d = np.full((X, Y), pal_size, np.int32)
    for q in rec.reshape(-1, 6):
        x, y = int(q[0]["p"][0]), int(q[0]["p"][1])
        w, h = int(q["d"][:, 0].max()), int(q["d"][:, 1].max())
        c2d[x:x + w, y:y + h] = int(q[0]["c"])
    return c2d


def mesh2d(c2d: np.ndarray, pal_size: int = 22) -> list:
    """Quads (x, y, w, h, colour, id) of sdf.cpp:367-397: per colour c < pal_size,
    cells visited x-major then y (forXY, voxmap.h:45-49); a quad grows along x
    while the mask holds (:378), then along y while the whole row of w cells
    holds (:380-385); its cells are cleared (:391-395); id 2 for glass =
    pal_size - 1 (:388)."""
    X, Y = c2d.shape
    quads = []
    for color in range(pal_size):
        mask = c2d == color
        if not mask.any():
            continue
        for x, y in np.argwhere(mask):          # row-major over (x, y) = forXY order
            x, y = int(x), int(y)
            if not mask[x, y]:
                continue
            w = 1
            while x + w < X and mask[x + w, y]:
                w += 1
            h = 1
            while y + h < Y and mask[x:x + w, y + h].all():
                h += 1
            quads.append((x, y, w, h, color, 2 if color == pal_size - 1 else 0))
            mask[x:x + w, y:y + h] = False
    return quads


def vertex2d_bytes(quads) -> bytes:
    """vert2d records (sdf.cpp:154-162: i16 x, y, 0, dx, dy, 0, u8 colour, 0, id, 0)
    of quad2d(x, y, w, 0, 0, h) = tri2d((0,0), (w,0), (0,h)) + tri2d((0,h), (w,0),
    (w,h)) (sdf.cpp:163-173, :389)."""
    out = np.zeros(6 * len(quads), REC2D)
    for k, (x, y, w, h, c, i) in enumerate(quads):
        for j, (dx, dy) in enumerate(((0, 0), (w, 0), (0, h), (0, h), (w, 0), (w, h))):
            out[6 * k + j] = ((x, y, 0), (dx, dy, 0), c, 0, i, 0)
    return out.tobytes()


def vertex_bytes(quads: np.ndarray) -> bytes:
    """vert records of the 3D mesh (sdf.cpp:94-141): quad() = tri(0, du, dv) +
    tri(dv, du, du + dv), each tri's last two vertices swapped for odd normals
    (:112-118, the winding GL culls by)."""
    rec = np.dtype([("p", "<i2", 3), ("d", "<i2", 3), ("c", "u1"), ("n", "u1"), ("id", "u1"), ("pad", "u1")])
    out = []
    for q in np.asarray(quads):
        o, du, dv = q[0:3], q[3:6], q[6:9]
        c, n, i = int(q[9]), int(q[10]), int(q[11])
        for a, b, cc in ((0 * du, du, dv), (dv, du, du + dv)):
            tri = (a, cc, b) if n % 2 else (a, b, cc)
            for d in tri:
                out.append(((int(o[0]), int(o[1]), int(o[2])), tuple(int(v) for v in d), c, n, i, 0))
    return np.array(out, rec).tobytes()
