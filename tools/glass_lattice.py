"""Cost of glass in draw order where many panes stack: glass_chain
re-walks the ray once per blended pane (glass_scan), so a pixel with P stacked
panes costs O(P^2) walk steps.  This builds a ground plane with a glass lattice
(sheets on every 4th x and y plane over a 256 x 128 block, 16 cells high) and times C3
full-quality frames of it at cameras K0-K2 in draw order (the default) and with
the single layer (VX_FLAG_GLASS_SINGLE), next to the plain S-proc frame, plus
the pane histogram (oracle glass_layers at 1/8 resolution, CPU).
usage: python tools/glass_lattice.py [--out gpurun_out/glass_lattice.json] [--no-gpu]"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def lattice():
    import numpy as np

    from voxmap_amd import scenes
    g = np.zeros((32, 256, 1024), np.uint8)
    g[0] = 2                                       # ground only: nothing hides the lattice
    g[1:20, 100:156, 700:720] = 9                  # one opaque block behind it
    x0, x1, y0, y1 = 384, 640, 64, 192
    blk = g[1:17, y0:y1, x0:x1]
    blk[:, :, ::4] = scenes.GLASS
    blk[:, ::4, :] = scenes.GLASS
    return g


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--no-gpu", action="store_true")
    ap.add_argument("--frames", type=int, default=20)
    args = ap.parse_args()
    import numpy as np

    import voxmap_amd as vx
    from voxmap_amd import presets, scenes
    noise = scenes.real_noise()
    res = {"scene": "ground + glass sheets on every 4th x and y plane of x 384..639, y 64..191, z 1..16, a block behind"}
    g = lattice()
    if args.no_gpu:
        import oracle
        field = vx.field_build(g)
        O = oracle.Oracle(field, noise)
        for cam in ("K0", "K1", "K2"):
            fr = presets.camera_frame(cam, 480, 270, flags=48)
            n = O.glass_layers(fr.params, 480, 270)
            h = np.bincount(n.ravel(), minlength=2)
            res[f"panes_{cam}"] = {"max": int(n.max()), "ge2_frac": float((n >= 2).mean()),
                                   "ge8_frac": float((n >= 8).mean()), "hist_head": h[:12].tolist()}
            print(cam, res[f"panes_{cam}"], flush=True)
    else:
        import torch
        torch.cuda.set_device(0)
        W, H = 3840, 2160
        out = torch.empty(W * H * 4, dtype=torch.uint8, device="cuda")
        for name, grid in (("lattice", g), ("s_proc", presets.scene_grid("s_proc"))):
            Z, Y, X = grid.shape
            with vx.Scene(map_bytes=grid.tobytes(), map_format=vx.FORMAT_GRID, noise_path=scenes.NOISE_PATH,
                          dims=(X, Y, Z), device=0) as sc:
                for cam in ("K0", "K1", "K2"):
                    for tag, fl in (("order", 48), ("single", 48 | vx.FLAG_GLASS_SINGLE)):
                        fr = presets.camera_frame(cam, W, H, flags=fl)
                        sc.prepare_sun(fr)
                        glass = sc.render_device(fr, out.data_ptr(), pixel_format=vx.PIXEL_RGBA8, stats=True).glass_px
                        st = torch.cuda.Stream()          # events and launches on one non-default stream
                        ms = []
                        for _ in range(7):          # median of 7 blocks of `frames` timed (non-STATS) launches
                            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                            e0.record(st)
                            for _ in range(args.frames):
                                sc.render_device(fr, out.data_ptr(), pixel_format=vx.PIXEL_RGBA8,
                                                 stream=st.cuda_stream)
                            e1.record(st)
                            torch.cuda.synchronize()
                            ms.append(e0.elapsed_time(e1) / args.frames)
                        res[f"{name}:{cam}:{tag}"] = {"ms": round(statistics.median(ms), 4), "glass_px": int(glass)}
                        print(name, cam, tag, res[f"{name}:{cam}:{tag}"], flush=True)
    if args.out:
        json.dump(res, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
