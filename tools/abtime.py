"""Interleaved A/B timing of library variants in ONE process on one GPU.

Each variant .so is loaded with ctypes side by side (distinct paths), gets its
own scene of the same grid, and renders the same frame into the same device
framebuffer; rounds alternate between variants so clock/thermal drift hits
all of them alike.  Reports the median ms per frame per variant and flags.

usage: python tools/abtime.py [--config C3] [--flags 0,48] [--rounds 7] [--frames 20] label=path.so[:cap][+orflags] ...
(+orflags: flags OR-ed into every frame of that variant, e.g. one library with
and without a diagnostic flag, interleaved: head=lib.so nodoom=lib.so+131072)
"""
from __future__ import annotations

import argparse
import ctypes as C
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--flags", default="0,48")
    ap.add_argument("--samples", type=int, default=None)
    ap.add_argument("--scene", default=None, help="override the config's scene (e.g. s_glass)")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--frames", type=int, default=20)
    ap.add_argument("variants", nargs="+")
    args = ap.parse_args()
    import torch

    from voxmap_amd import _abi, presets
    torch.cuda.set_device(0)
    cfg = presets.CONFIGS[args.config]
    grid = presets.scene_grid(args.scene or cfg["scene"])
    Z, Y, X = grid.shape
    W, H = cfg["w"], cfg["h"]
    up = 3.0 if cfg["scene"] == "s_up3" else 1.0
    samples = args.samples if args.samples is not None else cfg.get("samples", 1)
    gbytes = grid.tobytes()
    libs = []
    for spec in args.variants:
        label, path = spec.split("=", 1)
        orf = 0
        if "+" in path:                 # label=lib.so+FLAGS -- flags OR-ed into this variant's frames
            path, orf = path.rsplit("+", 1)
            orf = int(orf)
        cap = 0
        if ":" in path:                 # label=lib.so:CAP -- the scene's dist_cap (traversal box cap)
            path, cap = path.rsplit(":", 1)
            cap = int(cap)
        L = C.CDLL(os.path.abspath(path))
        for name, res, argt in _abi.SIGNATURES:
            try:
                fn = getattr(L, name)
            except AttributeError:      # an older ABI: only the symbols used here are needed
                continue
            fn.restype, fn.argtypes = res, argt
        d = _abi.SceneDesc()
        buf = C.create_string_buffer(gbytes, len(gbytes))
        d.map_bytes = C.cast(buf, C.c_void_p)
        d.map_size = len(gbytes)
        d.map_format = _abi.FORMAT_GRID
        d.X, d.Y, d.Z = X, Y, Z
        d.dist_cap = cap
        h = C.c_void_p()
        rc = L.vx_scene_create(C.byref(d), C.byref(h))
        if rc:
            raise SystemExit(f"{label}: {L.vx_last_error().decode()}")
        libs.append((label, L, h, orf))
    out = torch.empty(W * H * 4, dtype=torch.uint8, device="cuda")
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    res = {}
    for flags in [int(f) for f in args.flags.split(",")]:
        ps = {}
        for lab, _, _, orf in libs:
            ps[lab] = presets.camera_frame(cfg["camera"], W, H, scale=up, flags=flags | orf, shadow_samples=samples,
                                           sun_radius=0.03 if samples > 1 else 0.0).params
        times = {lab: [] for lab, _, _, _ in libs}
        for r in range(args.rounds + 1):
            for lab, L, h, _ in (libs if r % 2 == 0 else libs[::-1]):
                p = ps[lab]
                for _ in range(3):
                    L.vx_render(h, C.byref(p), W, H, _abi.PIXEL_RGBA8, C.c_void_p(out.data_ptr()), 1,
                                C.c_void_p(stream.cuda_stream), None)
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.frames):
                    L.vx_render(h, C.byref(p), W, H, _abi.PIXEL_RGBA8, C.c_void_p(out.data_ptr()), 1,
                                C.c_void_p(stream.cuda_stream), None)
                e1.record()
                torch.cuda.synchronize()
                if r > 0:                       # round 0 warms everything up
                    times[lab].append(e0.elapsed_time(e1) / args.frames)
        ref = None                          # every variant's frame against the first one's
        for lab, L, h, _ in libs:
            L.vx_render(h, C.byref(ps[lab]), W, H, _abi.PIXEL_RGBA8, C.c_void_p(out.data_ptr()), 1,
                        C.c_void_p(stream.cuda_stream), None)
            torch.cuda.synchronize()
            img = out.cpu()
            if ref is None:
                ref = img
            else:
                print(f"{args.config} flags={flags:3d} {lab:14s} {int((img != ref).sum())} bytes differ from "
                      f"{libs[0][0]}", flush=True)
        base = None
        for lab, _, _, _ in libs:
            med = statistics.median(times[lab])
            base = base or med
            res[(lab, flags)] = med
            print(f"{args.config} flags={flags:3d} {lab:14s} median {med:.4f} ms  ({100 * (med / base - 1):+.1f}%)  "
                  f"min {min(times[lab]):.4f}", flush=True)
    for lab, L, h, _ in libs:
        L.vx_scene_destroy(h)


if __name__ == "__main__":
    main()
