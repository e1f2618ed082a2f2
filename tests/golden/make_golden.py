"""Regenerate tests/golden/frames.npz — golden RGBA fp32 frames of the oracle.

Inputs are synthetic (the reference holds no golden images): small
S-proc-style scenes built by vx_field_build (sdf.cpp:405-470 restatement), the
A channel by the oracle's distance pass, synthetic noise seed 0.  Run from the
repo root:  python tests/golden/make_golden.py
"""
import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import oracle  # noqa: E402
import voxmap_amd as vx  # noqa: E402
from voxmap_amd import scenes  # noqa: E402

CASES = [
    {"name": "proc_oblique", "seed": 5, "dims": [96, 48, 16], "sbj": [48.0, 24.0, 18.0], "rot": [1.1, 0.0, 0.6]},
    {"name": "proc_top", "seed": 7, "dims": [96, 48, 16], "sbj": [48.0, 24.0, 40.0], "rot": [1e-4, 0.0, -0.002]},
    {"name": "proc_glass_grazing", "seed": 11, "dims": [128, 64, 24], "sbj": [-6.0, 32.0, 9.0],
     "rot": [1.45, 0.0, -1.5707963267948966], "n_glass": 12},
    # extensions (pinned to this build's own definition only)
    {"name": "ext_full_quality", "seed": 11, "dims": [128, 64, 24], "sbj": [-6.0, 32.0, 9.0],
     "rot": [1.45, 0.0, -1.5707963267948966], "n_glass": 12, "frame": {"flags": 48}},
    {"name": "ext_soft16", "seed": 5, "dims": [96, 48, 16], "sbj": [48.0, 24.0, 18.0], "rot": [1.1, 0.0, 0.6],
     "frame": {"flags": 48, "shadow_samples": 16, "sun_radius": 0.05}},
]
W, H = 64, 48


def inputs(case):
    g = scenes.small_proc(case["seed"], dims=tuple(case["dims"]), n_boxes=16, n_glass=case.get("n_glass", 6))
    field = vx.field_build(g)
    noise = vx.noise_synth(0)
    fr = vx.make_frame(tuple(case["sbj"]), tuple(case["rot"]), W, H, **case.get("frame", {}))
    return field, noise, fr


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


if __name__ == "__main__":
    out = {}
    meta = []
    for c in CASES:
        field, noise, fr = inputs(c)
        img, st = oracle.Oracle(field, noise).render(fr.params, W, H)
        out[c["name"]] = img
        meta.append({**c, "w": W, "h": H, "field_sha256": sha(field), "noise_sha256": sha(noise),
                     "params": vx.params_to_dict(fr.params), "stats": st.as_dict()})
    np.savez_compressed(os.path.join(os.path.dirname(__file__), "frames.npz"), **out)
    json.dump(meta, open(os.path.join(os.path.dirname(__file__), "frames.json"), "w"), indent=1)
    print("wrote", list(out))
