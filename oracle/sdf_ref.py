"""Pure-Python literal restatement of the field generator — TEST INFRASTRUCTURE.

Follows /root/reference/src/gen/sdf.cpp line by line for tiny grids (it is a
loop-for-loop transliteration, so only small dims finish quickly):
  csum() clamped sum access ............ sdf.cpp:36-42
  csdf() clamped sdf access ............ sdf.cpp:54-61
  vol() inclusive box count ............ sdf.cpp:63-83
  summed volume table, forXYZ .......... sdf.cpp:407-422
  half-cube radii with the mid shortcut  sdf.cpp:429-457
  map.bin texel order (R, G, B=col, A=0) sdf.cpp:462-470
  air remapped to B = pal_size ......... sdf.cpp:19,188,229-233
Arrays are zero-initialised like the reference's globals (sdf.cpp:22-25).
"""
from __future__ import annotations

import numpy as np

PAL_SIZE = 22   # render.vert:21 palette entries: 0 (air) + 20 colours + glass


def build(color_zyx: np.ndarray) -> np.ndarray:
    Z, Y, X = color_zyx.shape
    col = [[[int(color_zyx[z, y, x]) for z in range(Z)] for y in range(Y)] for x in range(X)]
    bin_ = [[[1 if col[x][y][z] else 0 for z in range(Z)] for y in range(Y)] for x in range(X)]
    sum_ = [[[0] * Z for _ in range(Y)] for _ in range(X)]
    sdf = [[[[0, 0] for _ in range(Z)] for _ in range(Y)] for _ in range(X)]

    def cl(v, hi):
        return 0 if v < 0 else (hi - 1 if v > hi - 1 else v)

    def csum(x, y, z):
        return sum_[cl(x, X)][cl(y, Y)][cl(z, Z)]

    def csdf(x, y, z, o):
        return sdf[cl(x, X)][cl(y, Y)][cl(z, Z)][o]

    def vol(x0, y0, z0, x1, y1, z1):
        x0 -= 1
        y0 -= 1
        z0 -= 1
        return (0 - csum(x1, y1, z0) - csum(x1, y0, z1) - csum(x0, y1, z1) + csum(x1, y1, z1)
                + csum(x0, y0, z1) + csum(x0, y1, z0) + csum(x1, y0, z0) - csum(x0, y0, z0))

    for x in range(X):
        for y in range(Y):
            for z in range(Z):
                sum_[x][y][z] = (bin_[x][y][z] + csum(x, y, z - 1) + csum(x, y - 1, z) + csum(x - 1, y, z)
                                 - csum(x - 1, y - 1, z) - csum(x - 1, y, z - 1) - csum(x, y - 1, z - 1)
                                 + csum(x - 1, y - 1, z - 1))
    for x in range(X):
        for y in range(Y):
            for z in range(Z):
                if bin_[x][y][z] > 0:
                    continue
                for o in range(2):
                    mn = 1
                    mx = Z if o == 0 else z
                    if x + y + z > 0:
                        mid = csdf(x - 1, y - 1, z - 1, o)
                        mn = max(mn, mid - 1)
                        mx = min(mx, mid + 1)
                    r = mn
                    while r < mx and vol(x - r, y - r, z - o * r, x + r, y + r, z + (1 - o) * r) == 0:
                        r += 1
                    sdf[x][y][z][o] = r
    out = np.zeros((Z, Y, X, 4), np.uint8)
    for z in range(Z):
        for y in range(Y):
            for x in range(X):
                # B = the remapped index: air (0) finds pal[pal_size] = 0 in the
                # zero-initialised pal[] scanned from 1 (sdf.cpp:19,188,229-233)
                b = col[x][y][z] if col[x][y][z] else PAL_SIZE
                out[z, y, x] = (sdf[x][y][z][0] & 0xFF, sdf[x][y][z][1] & 0xFF, b & 0xFF, 0)
    return out
