"""Work counters of one workload under two library builds (ctypes, one process):
prints each library's vx_stats for the same frame (diagnostic of a kernel change
that must keep the frame and the fetch counts and may change the wave counters).
usage: python tools/stats_ab.py [--config C3] [--flags 48] label=lib.so ..."""
import argparse
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--flags", type=int, default=48)
    ap.add_argument("variants", nargs="+")
    args = ap.parse_args()
    import torch

    from voxmap_amd import _abi, presets
    cfg = presets.CONFIGS[args.config]
    grid = presets.scene_grid(cfg["scene"])
    Z, Y, X = grid.shape
    W, H = cfg["w"], cfg["h"]
    samples = cfg.get("samples", 1)
    fr = presets.camera_frame(cfg["camera"], W, H, scale=3.0 if cfg["scene"] == "s_up3" else 1.0, flags=args.flags,
                              shadow_samples=samples, sun_radius=0.03 if samples > 1 else 0.0)
    gbytes = grid.tobytes()
    out = torch.empty(W * H * 4, dtype=torch.uint8, device="cuda")
    for spec in args.variants:
        label, path = spec.split("=", 1)
        L = C.CDLL(os.path.abspath(path))
        for name, res, argt in _abi.SIGNATURES:
            if hasattr(L, name):
                fn = getattr(L, name)
                fn.restype, fn.argtypes = res, argt
        d = _abi.SceneDesc()
        buf = C.create_string_buffer(gbytes, len(gbytes))
        d.map_bytes = C.cast(buf, C.c_void_p)
        d.map_size = len(gbytes)
        d.map_format = _abi.FORMAT_GRID
        d.X, d.Y, d.Z = X, Y, Z
        h = C.c_void_p()
        assert L.vx_scene_create(C.byref(d), C.byref(h)) == 0
        st = _abi.Stats()
        assert L.vx_render(h, C.byref(fr.params), W, H, _abi.PIXEL_RGBA8, C.c_void_p(out.data_ptr()), 1, None,
                           C.byref(st)) == 0
        torch.cuda.synchronize()
        dd = st.as_dict()
        print(label, {k: dd[k] for k in ("shadow_rays", "shadow_fetches", "march_wave_iters", "march_lane_slots",
                                        "primary_wave_iters", "kernel_ms")}, flush=True)
        L.vx_scene_destroy(h)


if __name__ == "__main__":
    main()
