"""Rasterise the reference's plaintext 2D mesh (res/vertex2d.bin.gz) into a
(256, 1024) top-colour map: voxmap_amd/data/campus_footprint.npy.gz.

Record layout (sdf.cpp:94-102 / :154-162 for vert2d, render.js:12): i16 x, y, z,
i16 dx, dy, dz, i8 colour, i8 normal, i8 id, pad — 16 bytes.  quad2d(x, y, w, 0,
0, h, colour) (sdf.cpp:169-173, :389) emits 6 vertices whose offsets span
[0,w] x [0,h]; each quad covers cells [x, x+w) x [y, y+h).
Run once in the build container (needs /root/reference); the output is data.
"""
import gzip
import io
import sys

import numpy as np

src = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/res/vertex2d.bin.gz"
dst = sys.argv[2] if len(sys.argv) > 2 else "voxmap_amd/data/campus_footprint.npy.gz"
raw = gzip.decompress(open(src, "rb").read())
rec = np.frombuffer(raw, dtype=np.dtype([("p", "<i2", 3), ("d", "<i2", 3), ("c", "i1"), ("n", "i1"),
                                         ("id", "i1"), ("pad", "i1")]))
assert len(rec) % 6 == 0, len(rec)
fp = np.zeros((256, 1024), np.uint8)
q = rec.reshape(-1, 6)
for quad in q:
    x, y = int(quad[0]["p"][0]), int(quad[0]["p"][1])
    w = int(max(v["d"][0] for v in quad)); h = int(max(v["d"][1] for v in quad))
    fp[y:y + h, x:x + w] = int(quad[0]["c"]) & 0xFF
buf = io.BytesIO()
np.save(buf, fp, allow_pickle=False)
with gzip.open(dst, "wb", compresslevel=9) as f:
    f.write(buf.getvalue())
print(dst, fp.shape, "quads", len(q), "colours", np.unique(fp))
