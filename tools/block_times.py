"""Per-block start/end times of one render launch (diagnostics build with
-DVX_BLOCK_TIMING, e.g. ab/lib_btime.so): how long the launch's tail is --
the time from the first block that finds no more work to the end -- and how
block durations spread over the frame.
usage: python tools/block_times.py lib.so [--config C5] [--flags 48] [--frames 5]"""
import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib")
    ap.add_argument("--config", default="C5")
    ap.add_argument("--flags", type=int, default=48)
    ap.add_argument("--frames", type=int, default=5)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    import numpy as np
    import torch
    from voxmap_amd import _abi, presets, scenes
    torch.cuda.set_device(0)
    L = C.CDLL(os.path.abspath(args.lib))
    for name, res, argt in _abi.SIGNATURES:
        fn = getattr(L, name)
        fn.restype, fn.argtypes = res, argt
    L.vx_debug_block_times.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.POINTER(C.c_size_t)]
    cfg = presets.CONFIGS[args.config]
    grid = presets.scene_grid(cfg["scene"])
    Z, Y, X = grid.shape
    W, H = cfg["w"], cfg["h"]
    up = 3.0 if cfg["scene"] == "s_up3" else 1.0
    samples = cfg.get("samples", 1)
    d = _abi.SceneDesc()
    gb = grid.tobytes()
    buf = C.create_string_buffer(gb, len(gb))
    d.map_bytes, d.map_size, d.map_format = C.cast(buf, C.c_void_p), len(gb), _abi.FORMAT_GRID
    d.noise_path = scenes.NOISE_PATH.encode()
    d.X, d.Y, d.Z = X, Y, Z
    h = C.c_void_p()
    assert L.vx_scene_create(C.byref(d), C.byref(h)) == 0, L.vx_last_error()
    fr = presets.camera_frame(cfg["camera"], W, H, scale=up, flags=args.flags, shadow_samples=samples,
                              sun_radius=0.03 if samples > 1 else 0.0)
    out = torch.empty(W * H * 4, dtype=torch.uint8, device="cuda")
    res = []
    for f in range(args.frames + 2):
        assert L.vx_render(h, C.byref(fr.params), W, H, 1, C.c_void_p(out.data_ptr()), 1, None, None) == 0
        torch.cuda.synchronize()
        n = C.c_size_t()
        L.vx_debug_block_times(h, None, 0, C.byref(n))
        t = np.zeros(2 * n.value, np.uint64)
        L.vx_debug_block_times(h, t.ctypes.data, t.size, C.byref(n))
        if f < 2:
            continue
        t = t.reshape(-1, 2).astype(np.int64)
        t0 = t[:, 0].min()
        st, en = (t[:, 0] - t0) * 10.0, (t[:, 1] - t0) * 10.0          # ns
        dur = en - st
        span = en.max()
        # the tail: from the last block start to the launch end
        last_start = st.max()
        nb = len(st)
        bx = (W + 31) // 32
        rows = dur.reshape(-1, bx)
        res.append({"launch_us": round(span / 1e3, 2), "blocks": int(nb),
                    "mean_block_us": round(float(dur.mean()) / 1e3, 2),
                    "p50_block_us": round(float(np.percentile(dur, 50)) / 1e3, 2),
                    "p99_block_us": round(float(np.percentile(dur, 99)) / 1e3, 2),
                    "max_block_us": round(float(dur.max()) / 1e3, 2),
                    "last_start_us": round(float(last_start) / 1e3, 2),
                    "tail_us": round(float(span - last_start) / 1e3, 2),
                    "busy_frac": round(float(dur.sum()) / (span * 2048), 4),
                    "row_mean_us": [round(float(v) / 1e3, 1) for v in rows.mean(axis=1)[::10]]})
    print(json.dumps({"config": args.config, "flags": args.flags, "frames": res}, indent=1))
    if args.out:
        json.dump({"config": args.config, "flags": args.flags, "frames": res}, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
