"""Lockstep soft-shadow marches with a per-march step budget (a cost model, CPU only).

The oracle records the fetch count of every sun march of sampled 32x8 blocks
(vxo_march_lengths, with the build's exit tables).  Per wave (8x8 tile) the
kernel's lockstep loop costs sum_k (max over lanes of the k-th march + setup)
wave steps.  With a budget B, a march still running after B steps would leave
the wave (its state queued for a second pass); the wave then costs
sum_k (min(max_k, B) + setup) and the queued remainders sum(L - B) lane steps.
Prints, per B, the share of the frame's lockstep wave steps kept in the main
pass, the queued lane steps (in wave steps at full lanes), how many marches and
pixels spill, and the longest wave chain (the launch's critical path) before/after.
usage: python tools/march_spill.py [--config C5] [--blocks 120]
"""
from __future__ import annotations

import argparse
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C5")
    ap.add_argument("--blocks", type=int, default=120)
    ap.add_argument("--setup", type=float, default=0.7)
    args = ap.parse_args()
    import oracle
    import voxmap_amd as vx
    from voxmap_amd import presets, scenes
    cfg = presets.CONFIGS[args.config]
    grid = presets.scene_grid(cfg["scene"])
    field = vx.field_build(grid)
    W, H = cfg["w"], cfg["h"]
    samples = cfg.get("samples", 1)
    up = 3.0 if cfg["scene"] == "s_up3" else 1.0
    fr = presets.camera_frame(cfg["camera"], W, H, scale=up, flags=vx.FLAG_FULL_QUALITY, shadow_samples=samples,
                              sun_radius=0.03 if samples > 1 else 0.0)
    o = oracle.Oracle(field, scenes.real_noise(), exit=True)
    o.hold_exit_table(fr.params)
    L = oracle.lib()
    L.vxo_march_lengths.argtypes = [C.POINTER(oracle.OScene), C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int,
                                    C.c_int, C.c_int, C.c_void_p, C.c_int]
    L.vxo_march_lengths.restype = None
    maxrec = 2 * max(samples, 1) + 2
    rng = np.random.default_rng(11)
    waves = []
    for _ in range(args.blocks):
        px0 = int(rng.integers(0, W // 32)) * 32
        py0 = int(rng.integers(0, H // 8)) * 8
        buf = np.empty((8, 32, maxrec), np.int32)
        L.vxo_march_lengths(C.byref(o.sc), C.addressof(fr.params), W, H, px0, py0, 32, 8, buf.ctypes.data, maxrec)
        for w in range(4):
            t = buf[:, 8 * w:8 * w + 8].reshape(64, maxrec)
            waves.append(np.where(t >= 0, t & 0xFFFF, -1))
    tot_lock = 0.0
    chains = []
    for t in waves:
        c = sum(t[:, k].max() + args.setup for k in range(t.shape[1]) if (t[:, k] >= 0).any())
        chains.append(c)
        tot_lock += c
    chains = np.array(chains)
    allm = np.concatenate([t[t >= 0] for t in waves])
    print(f"{args.config} camera scale {up}: {len(waves)} waves, {allm.size} marches, mean length {allm.mean():.2f}, "
          f"p99 {np.percentile(allm, 99):.0f}, max {allm.max()}")
    print(f"  lockstep wave chains: mean {chains.mean():.1f}  p50 {np.percentile(chains, 50):.1f}  "
          f"p99 {np.percentile(chains, 99):.1f}  max {chains.max():.1f} wave steps")
    per_wave = {}
    for B in (8, 12, 16, 20, 24, 32):
        kept, spill_steps, n_sp, px_sp, ch = 0.0, 0, 0, 0, []
        for t in waves:
            c = 0.0
            for k in range(t.shape[1]):
                col = t[:, k]
                if (col >= 0).any():
                    c += min(col.max(), B) + args.setup
            kept += c
            ch.append(c)
            s = t[t > B]
            per_wave.setdefault(B, []).append(s.size)
            spill_steps += int((s - B).sum())
            n_sp += s.size
            px_sp += int((t > B).any(axis=1).sum())
        print(f"  B={B:3d}: main pass {kept / tot_lock:.3f} of lockstep, queued {spill_steps / 64 / tot_lock:.3f} "
              f"(at full lanes), spilled marches {n_sp / allm.size:.4f}, pixels {px_sp / (64 * len(waves)):.4f}, "
              f"longest wave chain {max(ch):.0f}; queued per wave p50/p99/max "
              f"{np.percentile(per_wave[B], 50):.0f}/{np.percentile(per_wave[B], 99):.0f}/{max(per_wave[B])}")


if __name__ == "__main__":
    main()
