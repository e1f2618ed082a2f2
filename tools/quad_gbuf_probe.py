"""How much the G-buffer split changes the frame.

The raster hands render.frag a flat v_cellPos = the greedy quad's origin and a
smooth v_fractPos that spans the quad (render.vert:25-28; records sdf.cpp:94-141,
quads :284-356).  The unit-cell split starts every fragment from the hit cell
instead.  Both are the same point; the fp32 split differs, and main() feeds it
to rayDir (render.frag:154), the AO sample (:223) and the sun march (:233,
whose first step takes fract(-f*sign(r)) of an f up to ~CHUNK).

Per BASELINE frame this renders the oracle in both modes and counts the pixels
whose sun-march lit flag differs, whose AO distance differs, whose fp32 RGBA
differs at all and beyond 1e-5 relative, and whose RGBA8 differs.
usage: python tools/quad_gbuf_probe.py [--frames C2:K0,C2:K1,C2:K2,C3:K1:v1,C3:K1:full] [--out path]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", default="C2:K0:v1,C2:K1:v1,C2:K2:v1,C3:K1:v1,C3:K1:full")
    ap.add_argument("--threads", type=int, default=0)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    import numpy as np

    import oracle
    import voxmap_amd as vx
    from voxmap_amd import presets, scenes

    noise = scenes.real_noise()
    cache = {}
    res = {}
    for spec in args.frames.split(","):
        cfg, cam, q = spec.split(":")
        c = presets.CONFIGS[cfg]
        if c["scene"] not in cache:
            field = vx.field_build(presets.scene_grid(c["scene"]))
            t0 = time.time()
            qoff = oracle.face_quads(field)
            tq = time.time() - t0
            cache[c["scene"]] = (oracle.Oracle(field, noise, exit=True),
                                 oracle.Oracle(field, noise, exit=True, quad=qoff), tq)
        unit, quad, tq = cache[c["scene"]]
        flags = vx.FLAG_FULL_QUALITY if q == "full" else 0
        fr = presets.camera_frame(cam, c["w"], c["h"], flags=flags)
        h, w = c["h"], c["w"]
        ia, sa = unit.render(fr.params, w, h, threads=args.threads)
        ib, sb = quad.render(fr.params, w, h, threads=args.threads)
        la, aa = unit.terms(fr.params, w, h, threads=args.threads)
        lb, ab = quad.terms(fr.params, w, h, threads=args.threads)
        lit_diff = np.any(la != lb, axis=2)
        amb_diff = np.any((aa.view(np.uint32) != ab.view(np.uint32)) & ~(np.isnan(aa) & np.isnan(ab)), axis=2)
        word = ia.view(np.uint32) != ib.view(np.uint32)
        rel = np.abs(ia - ib) > 1e-5 * np.maximum(np.abs(ia), 1e-6)
        q8 = lambda im: np.floor(np.clip(im, 0, 1) * 255 + 0.5).astype(np.uint8)
        rgba8 = np.any(q8(ia) != q8(ib), axis=2)
        # lit -> unlit / unlit -> lit among the marched fragments of slot 0
        m = (la[..., 0] != 255) & (lb[..., 0] != 255)
        res[spec] = {
            "pixels": w * h,
            "block_px": int(sa.block_px), "glass_px": int(sa.glass_px),
            "lit_flag_differs": int(lit_diff.sum()),
            "lit_to_unlit": int((m & (la[..., 0] > lb[..., 0])).sum()),
            "unlit_to_lit": int((m & (la[..., 0] < lb[..., 0])).sum()),
            "ao_differs": int(amb_diff.sum()),
            "fp32_any_word_differs": int(np.any(word, axis=2).sum()),
            "fp32_beyond_1e-5": int(np.any(rel, axis=2).sum()),
            "rgba8_differs": int(rgba8.sum()),
            "shadow_fetches_unit_quad": [int(sa.shadow_fetches), int(sb.shadow_fetches)],
        }
        print(spec, json.dumps(res[spec]), flush=True)
    out = {"what": "oracle frames with the unit-cell G-buffer vs the quad-relative one (v_cellPos = greedy quad "
                   "origin, v_fractPos = hit - origin in fp32, render.vert:25-28); exit tables on (frames are "
                   "identical with and without them)",
           "face_quads_s": {k: round(v[2], 3) for k, v in cache.items()}, "frames": res}
    if args.out:
        with open(args.out, "w") as f:
            json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
