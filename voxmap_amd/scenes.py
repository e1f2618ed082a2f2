"""Synthetic scenes in the reference's map.bin format.

The real field (res/map.blob) is AES-encrypted with a key that is not in the
reference repository (src/web/ui.js:47,169-179), so benchmarks and parity
tests run on synthetic palette-index grids with the same layout, turned into
map.bin texels by ``vx_field_build`` (the sdf.cpp:405-470 restatement).

Grids are (Z, Y, X) uint8 palette indices, x fastest in memory like map.bin
(render.js:62).  Index 0 = air, 1..20 = opaque palette colours, 21 = glass
(render.vert:21, sdf.cpp:195,337).
"""
from __future__ import annotations

import gzip
import os

import numpy as np

GLASS = 21
_DATA = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data")


def s_proc(seed: int = 1, dims=(1024, 256, 32), n_boxes: int = 400, n_glass: int = 30) -> np.ndarray:
    """S-proc: ground, ~400 boxes (w 4-40, h 2-28, palette 1-20), ~5% overhang
    slabs, 30 glass panes.  Deterministic in ``seed``."""
    X, Y, Z = dims
    rng = np.random.default_rng(seed)
    g = np.zeros((Z, Y, X), np.uint8)
    g[0] = 2                                   # grass ground at z = 0
    # a few roads / courtyards on the ground plane
    for _ in range(max(1, X // 64)):
        if rng.random() < 0.5:
            y0 = int(rng.integers(0, Y - 8)); g[0, y0:y0 + int(rng.integers(3, 8)), :] = 13
        else:
            x0 = int(rng.integers(0, X - 8)); g[0, :, x0:x0 + int(rng.integers(3, 8))] = 13
    zmax = Z - 1
    for _ in range(n_boxes):
        w = int(rng.integers(4, 41)); d = int(rng.integers(4, 41))
        hgt = int(rng.integers(2, min(29, zmax) + 1))
        x0 = int(rng.integers(0, max(1, X - w))); y0 = int(rng.integers(0, max(1, Y - d)))
        col = int(rng.integers(1, 21))
        if rng.random() < 0.05:                # overhang slab: floating roof with air beneath
            z0 = int(rng.integers(3, max(4, zmax - 3)))
            t = int(rng.integers(1, 4))
            g[z0:min(Z, z0 + t), y0:y0 + d, x0:x0 + w] = col
            # one supporting pillar so it reads as a building
            g[1:z0, y0:y0 + 2, x0:x0 + 2] = col
        else:
            g[1:1 + hgt, y0:y0 + d, x0:x0 + w] = col
    for _ in range(n_glass):                   # glass panes, 1 voxel thick
        L = int(rng.integers(6, 30)); hgt = int(rng.integers(3, min(20, zmax)))
        x0 = int(rng.integers(0, X - L)); y0 = int(rng.integers(0, Y - L))
        if rng.random() < 0.5:
            g[1:1 + hgt, y0, x0:x0 + L] = GLASS
        else:
            g[1:1 + hgt, y0:y0 + L, x0] = GLASS
    return g


# colour -> storey height for the campus extrusion (deterministic, arbitrary:
# the plaintext vertex2d.bin.gz carries top colours but no heights, sdf.cpp:156)
_CAMPUS_HEIGHT = np.array([0, 1, 1, 6, 9, 12, 8, 7, 5, 1, 1, 10, 14, 4, 3, 11, 13, 6, 9, 16, 2, 8], np.int32)


NOISE_PATH = os.path.join(_DATA, "noise.bin.gz")


def real_noise() -> np.ndarray:
    """(1024, 1024, 4) RGBA8: the reference's plaintext res/noise.bin.gz
    (noise.cpp:34-41 layout; render.js:138-149 uploads it as u_noise),
    shipped as data in voxmap_amd/data/."""
    with gzip.open(NOISE_PATH, "rb") as f:
        return np.frombuffer(f.read(), np.uint8).reshape(1024, 1024, 4)


def campus_footprint() -> np.ndarray:
    """(Y, X) top-colour map rasterised from the reference's plaintext
    res/vertex2d.bin.gz by tools/make_campus_footprint.py."""
    path = os.path.join(_DATA, "campus_footprint.npy.gz")
    with gzip.open(path, "rb") as f:
        return np.load(f, allow_pickle=False)


def s_campus(dims=(1024, 256, 32)) -> np.ndarray:
    """S-campus: the real campus footprint extruded by a fixed colour->height table."""
    X, Y, Z = dims
    fp = campus_footprint()
    assert fp.shape == (Y, X), fp.shape
    g = np.zeros((Z, Y, X), np.uint8)
    g[0] = np.where(fp > 0, fp, 2).astype(np.uint8)
    hgt = _CAMPUS_HEIGHT[np.minimum(fp, 21)]
    hgt = np.minimum(hgt, Z - 1)
    for z in range(1, Z):
        m = hgt >= z
        g[z][m] = fp[m]
    return g


def upsample3(g: np.ndarray, k: int = 3) -> np.ndarray:
    """S-up3: nearest k-fold upsample (C5's 3072x768x96 field)."""
    return np.repeat(np.repeat(np.repeat(g, k, axis=0), k, axis=1), k, axis=2)


def s_glass(seed: int = 1, dims=(1024, 256, 32), n_houses: int = 60, n_facades: int = 40) -> np.ndarray:
    """S-glass: S-proc plus glass that stacks along a view ray (the
    single-layer deviation): hollow glass pavilions (a one-voxel glass shell
    around air: a ray crosses the front pane, then the inside of the back pane,
    both front-facing glass faces) and glass screens standing off two facades of
    a building.  Deterministic in ``seed``."""
    X, Y, Z = dims
    g = s_proc(seed, dims)
    rng = np.random.default_rng(seed + 1000)
    for _ in range(n_houses):                  # hollow glass pavilions on the ground
        w = int(rng.integers(6, 24)); d = int(rng.integers(6, 24)); hgt = int(rng.integers(4, min(16, Z - 2)))
        x0 = int(rng.integers(0, X - w)); y0 = int(rng.integers(0, Y - d))
        g[1:1 + hgt, y0:y0 + d, x0:x0 + w] = GLASS
        g[1:hgt, y0 + 1:y0 + d - 1, x0 + 1:x0 + w - 1] = 0          # open inside, glass roof kept
    for _ in range(n_facades):                 # a building with glass screens off two facades
        w = int(rng.integers(8, 30)); d = int(rng.integers(8, 30)); hgt = int(rng.integers(6, min(24, Z - 1)))
        x0 = int(rng.integers(4, X - w - 4)); y0 = int(rng.integers(4, Y - d - 4))
        col = int(rng.integers(1, 21))
        g[1:1 + hgt, y0:y0 + d, x0:x0 + w] = col
        off = int(rng.integers(2, 4))
        g[1:1 + hgt, y0 - off, x0:x0 + w] = GLASS                  # screen in front of the -y facade
        g[1:1 + hgt, y0:y0 + d, x0 + w - 1 + off] = GLASS          # and of the +x facade
    return g


def single_block(dims=(64, 32, 16), at=(20, 12, 1), color=5) -> np.ndarray:
    X, Y, Z = dims
    g = np.zeros((Z, Y, X), np.uint8)
    g[0] = 2
    x, y, z = at
    g[z, y, x] = color
    return g


def glass_wall(dims=(64, 64, 16)) -> np.ndarray:
    """A glass wall (x = 36) over a ground plane with a white block behind it:
    looking up through the wall toward the sun (hour 1.0), the panes blend over
    cloudy sky next to the sun disc whose red exceeds 1 (render.frag:193,202:
    clouds mix toward sunCol.r = 1.4) and, with REFLECT, mirror it at grazing
    angles -- the case where the GL blend stage's clamps and 8-bit destination
    (render.js:84-86, map.js:7) decide the pixel (tests/golden 'blend_bright')."""
    X, Y, Z = dims
    g = np.zeros((Z, Y, X), np.uint8)
    g[0] = 2
    g[1:Z - 1, 4:Y - 4, 36] = GLASS
    g[1:6, 10:20, 50:56] = 20
    return g


def small_proc(seed: int, dims=(96, 48, 16), n_boxes=12, n_glass=3) -> np.ndarray:
    """A small S-proc-like scene that the scalar oracle renders in seconds."""
    return s_proc(seed, dims, n_boxes=n_boxes, n_glass=n_glass)
