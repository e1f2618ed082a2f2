"""Bands (the multi-GPU deal's kernel instantiation, TILED) against the whole
frame (untiled) on one GPU: the same C3 frame, every band, in place, RGBA8, one
stream; and a rank's share of the bands for N = 2, 4, 8 (diagnostics, GPU).
usage: python tools/band_time.py [--config C3] [--flags 48] [--frames 20]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--flags", type=int, default=48)
    ap.add_argument("--frames", type=int, default=20)
    ap.add_argument("--n", type=int, default=0, help="only this rank count (0: whole frame and 1, 2, 4, 8)")
    args = ap.parse_args()
    import numpy as np
    import torch

    import voxmap_amd as vx
    from voxmap_amd import dist, presets, scenes
    cfg = presets.CONFIGS[args.config]
    W, H = cfg["w"], cfg["h"]
    grid = presets.scene_grid(cfg["scene"])
    Z, Y, X = grid.shape
    fr = presets.camera_frame(cfg["camera"], W, H, flags=args.flags)
    out = torch.zeros(W * H * 4, dtype=torch.uint8, device="cuda")
    s = torch.cuda.Stream()
    with vx.Scene(map_bytes=grid.tobytes(), map_format=vx.FORMAT_GRID, noise_path=scenes.NOISE_PATH,
                  dims=(X, Y, Z), device=0) as sc:
        def timed(fn):
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            best = []
            for _ in range(5):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                for _ in range(args.frames):
                    fn()
                e1.record(s)
                torch.cuda.synchronize()
                best.append(e0.elapsed_time(e1) / args.frames)
            return float(np.median(best))
        if args.n:
            br = dist.band_rows_for(H, args.n)
            ids = list(range(0, -(-H // br), args.n))
            timed(lambda: sc.render_bands(fr, br, ids, out.data_ptr(), pixel_format=vx.PIXEL_RGBA8, stream=s.cuda_stream))
            print(f"N={args.n}: {br}-row bands, rank 0 renders {len(ids)} bands")
            return
        full = timed(lambda: sc.render_device(fr, out.data_ptr(), pixel_format=vx.PIXEL_RGBA8, stream=s.cuda_stream))
        ref = out.cpu().numpy().copy()
        print(f"{args.config} flags={args.flags} whole frame (untiled) {full:.4f} ms")
        for n in (1, 2, 4, 8):
            br = dist.band_rows_for(H, n)
            nb = -(-H // br)
            ids = list(range(0, nb, n))          # rank 0's bands
            t = timed(lambda: sc.render_bands(fr, br, ids, out.data_ptr(), pixel_format=vx.PIXEL_RGBA8,
                                              stream=s.cuda_stream))
            rows = sum(min(br, H - b * br) for b in ids)
            print(f"  N={n}: {br}-row bands, rank 0 renders {len(ids)} bands ({rows} rows): {t:.4f} ms "
                  f"= {t / full * H / rows:.3f} x the whole frame's time per row")
            if n == 1:
                assert np.array_equal(out.cpu().numpy(), ref), "bands differ from the whole frame"


if __name__ == "__main__":
    main()
