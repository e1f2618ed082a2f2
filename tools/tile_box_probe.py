"""How often the 64 rays of a wave tile (8x8 pixels) enter the grid inside the
air box of one corner ray's entry cell (a wave-uniform
first box read by a scalar load).  numpy restatement of the slab entry in
float64; boxes from oracle.field_box.  usage: python tools/tile_box_probe.py"""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, oracle, voxmap_amd as vx  # noqa: E402
from voxmap_amd import presets
field = vx.field_build(presets.scene_grid('s_proc'))
Z, Y, X, _ = field.shape
W, H = 3840, 2160
for cam in ("K1", "K0", "K2"):
    fr = presets.camera_frame(cam, W, H, flags=48)
    p = fr.params
    fwd, right, up = (np.array(getattr(p, k)[:], np.float64) for k in ("ray_fwd", "ray_right", "ray_up"))
    o = np.array(p.cam_cell[:], np.float64) + np.array(p.cam_fract[:], np.float64)
    px, py = np.meshgrid(np.arange(W), np.arange(H))
    nx = (2 * px + 1) / W - 1; ny = 1 - (2 * py + 1) / H
    d = fwd[None, None] + nx[..., None] * right[None, None] + ny[..., None] * up[None, None]
    dims = np.array([X, Y, Z], np.float64)
    with np.errstate(divide='ignore', invalid='ignore'):
        t0 = (0 - o) / d; t1 = (dims - o) / d
    tlo = np.max(np.minimum(t0, t1), axis=2).clip(min=0); thi = np.min(np.maximum(t0, t1), axis=2)
    hit = tlo < thi
    e = np.floor(o + tlo[..., None] * d).astype(np.int64)
    e = np.clip(e, 0, dims.astype(np.int64) - 1)
    oct = (d[..., 0] < 0) * 1 + (d[..., 1] < 0) * 2 + (d[..., 2] < 0) * 4
    boxes = {k: oracle.field_box(field, k) for k in np.unique(oct)}
    TY, TX = H // 8, W // 8
    ok_tiles = 0; tiles = 0; inside_px = 0
    for ty in range(TY):
        for tx in range(TX):
            sl = (slice(8 * ty, 8 * ty + 8), slice(8 * tx, 8 * tx + 8))
            h_ = hit[sl]
            if not h_.any():
                continue
            tiles += 1
            oc = oct[sl]
            best = 0
            for r in ((8 * ty, 8 * tx), (8 * ty, 8 * tx + 7), (8 * ty + 7, 8 * tx), (8 * ty + 7, 8 * tx + 7), (8*ty+3, 8*tx+3)):
                if not hit[r] or (oc != oct[r]).any():
                    continue
                c = e[r]; E = boxes[oct[r]][c[2], c[1], c[0]].astype(np.int64)
                s = np.where(d[r] >= 0, 1, -1)
                lo = np.where(s > 0, c, c - E); hi = np.where(s > 0, c + E, c)
                ee = e[sl]
                ins = np.all((ee >= lo) & (ee <= hi), axis=2) | ~h_
                best = max(best, int(ins[h_].sum()))
                if ins.all():
                    break
            inside_px += best
            if best == int(h_.sum()):
                ok_tiles += 1
    print(cam, "tiles with a hit", tiles, "all lanes inside the ref box", ok_tiles, round(ok_tiles / max(tiles, 1), 3),
          "pixels inside", round(inside_px / hit.sum(), 3), "camera", o)
