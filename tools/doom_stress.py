"""Stress of the sun doom table's stop rule (DESIGN.md §3 "Doom table") on the
oracle: adversarial scenes (sparse random voxels, one-cell-thick floating
roofs and poles, lattices) over ground, random suns (elevation 14-85 deg, every
azimuth), hard shadows and 2-16 soft samples, radii 0.005-0.06, default and short step budgets,
random cameras; every frame with the table must equal the frame without it
(VX_FLAG_NO_DOOM) word for word.  CPU only (test infrastructure).
usage: python tools/doom_stress.py SEED SCENES [Z (default 40)]"""
import os
import sys, math, time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import oracle
import voxmap_amd as vx
from voxmap_amd import scenes
noise = scenes.real_noise()
rng = np.random.default_rng(int(sys.argv[1]) if len(sys.argv) > 1 else 0)
NO_DOOM = 0x20000
bad = 0; tot = 0; saved = 0; allf = 0
t0 = time.time()
for it in range(int(sys.argv[2]) if len(sys.argv) > 2 else 6):
    X, Y, Z = 96, 64, int(sys.argv[3]) if len(sys.argv) > 3 else 40
    g = np.zeros((Z, Y, X), np.uint8)
    kind = it % 3
    if kind == 0:    # sparse random voxels
        g[2:] = (rng.random((Z - 2, Y, X)) < rng.uniform(0.03, 0.2)) * rng.integers(1, 20, (Z - 2, Y, X))
    elif kind == 1:  # thin floating slabs and poles
        for _ in range(60):
            x0, y0, z0 = rng.integers(0, X), rng.integers(0, Y), rng.integers(3, Z)
            w, h = rng.integers(1, 20), rng.integers(1, 20)
            if rng.random() < 0.5:
                g[z0, y0:y0 + h, x0:x0 + w] = rng.integers(1, 20)     # 1-cell-thick roof
            else:
                g[z0:min(Z, z0 + rng.integers(2, 15)), y0, x0] = rng.integers(1, 20)   # 1-cell pole
    else:            # checkerboard-ish lattices
        p = rng.integers(2, 5)
        g[4:, ::p, ::p] = (rng.random((Z - 4, (Y + p - 1) // p, (X + p - 1) // p)) < 0.4) * 7
    g[0] = 3                                                     # ground
    field = vx.field_build(g)
    o = oracle.Oracle(field, noise, exit=True)
    for k in range(8):
        el = rng.uniform(14, 85); az = rng.uniform(0, 360)
        er, ar = math.radians(el), math.radians(az)
        sun = (math.cos(er) * math.cos(ar), math.cos(er) * math.sin(ar), math.sin(er))
        n = int(rng.choice([1, 1, 2, 4, 8, 16])); rad = rng.uniform(0.005, 0.06) if n > 1 else 0.0
        maxs = int(rng.choice([0, 0, 20, 40]))
        cam = (rng.uniform(10, 86), rng.uniform(10, 54), rng.uniform(20, 39))
        rot = (rng.uniform(0.6, 1.4), 0.0, rng.uniform(-3, 3))
        res = []
        for fl in (0, NO_DOOM):
            fr = vx.make_frame(cam, rot, 96, 64, sun=sun, flags=48 | fl, shadow_samples=n, sun_radius=rad,
                               max_shadow_steps=maxs)
            img, st = o.render(fr.params, 96, 64)
            res.append((img, st.as_dict()["shadow_fetches"]))
        tot += 1
        same = np.array_equal(res[0][0].view(np.uint32), res[1][0].view(np.uint32))
        if not same:
            bad += 1
            print("DIFF", it, kind, k, el, az, n, rad, maxs, int((res[0][0] != res[1][0]).any(axis=2).sum()), flush=True)
        saved += res[1][1] - res[0][1]; allf += res[1][1]
    print(f"scene {it} kind {kind}: frames {tot} differing {bad}", flush=True)
print(f"frames {tot} differing {bad} fetches saved {saved} of {allf} in {time.time()-t0:.0f}s", flush=True)
