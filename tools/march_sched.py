"""Wave schedules of the soft-shadow marches (a cost model, CPU only).

The oracle records, per pixel of sampled 8x8 tiles (one wave64 each), the
fetch count of every sun march its shading runs (vxo_march_lengths, with the
build's exit tables).  Three schedules of a wave's marches are compared, in
wave steps:
  lockstep   the kernel's loop: sample k of every lane together; a wave step
             per step of the longest lane, plus a fixed setup per sample;
  refill     a lane starts its next march as soon as its march ends; a refill
             step costs the whole wave `--setup` steps, and runs when at least
             `--threshold` lanes wait (or every lane is waiting);
  ideal      no idle lanes: the total fetches / 64.
usage: python tools/march_sched.py [--config C3] [--samples 16] [--tiles 200]
"""
from __future__ import annotations

import argparse
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def lockstep(L, setup):
    """L: (64, m) fetch counts (-1 = no march); every lane runs its k-th march together."""
    cost = 0.0
    for k in range(L.shape[1]):
        col = L[:, k]
        if (col >= 0).any():
            cost += col.max() + setup
    return cost


def sorted_pool(L, setup, group, pool_setup):
    """Sample 0 of every lane in lockstep, then the remaining samples of the
    marching fragments dealt in pooled passes of 64 // group fragments x group
    lanes, fragments sorted by their sample-0 length (longest first): a pass
    costs its longest march + pool_setup (the per-pass state reload)."""
    cost = 0.0
    col = L[:, 0]
    if not (col >= 0).any():
        return 0.0
    cost += col.max() + setup
    frags = [r for r in L if r[0] >= 0]
    frags.sort(key=lambda r: -int(r[0]))
    per = 64 // group
    for i in range(0, len(frags), per):
        rest = np.concatenate([r[1:][r[1:] >= 0] for r in frags[i:i + per]] + [np.zeros(0, np.int64)])
        if rest.size:
            cost += rest.max() + pool_setup
    return cost


def block_classes(L, setup, pool_setup):
    """A 32x8 block (4 waves, L: (256, m)): sample 0 in lockstep per wave, then
    every remaining march of the block dealt 64 at a time over the 4 waves,
    the marches of fragments whose sample 0 ended unlit first (sorted by that
    length), so a pass holds marches of one class: wave steps summed over the
    block's waves."""
    cost = 0.0
    for w in range(4):
        col = L[64 * w:64 * (w + 1), 0]
        if (col >= 0).any():
            cost += col.max() + setup
    rest = []
    for r in L:
        if r[0] < 0:
            continue
        key = int(r[0])
        rest += [(key, int(v)) for v in r[1:] if v >= 0]
    rest.sort(key=lambda kv: -kv[0])
    for i in range(0, len(rest), 64):
        cost += max(v for _, v in rest[i:i + 64]) + pool_setup
    return cost


def refill(L, setup, threshold):
    queues = [list(r[r >= 0]) for r in L]
    cur = [q.pop(0) if q else -1 for q in queues]        # remaining steps of the running march
    cost = setup if any(c >= 0 for c in cur) else 0.0
    while True:
        active = [c for c in cur if c > 0]
        waiting = [i for i, c in enumerate(cur) if c <= 0 and queues[i]]
        if not active and not waiting:
            return cost
        if waiting and (len(waiting) >= threshold or not active):
            for i in waiting:
                cur[i] = queues[i].pop(0)
            cost += setup
            continue
        cost += 1
        cur = [c - 1 if c > 0 else c for c in cur]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--samples", type=int, default=16)
    ap.add_argument("--tiles", type=int, default=200)
    ap.add_argument("--setup", type=float, default=0.7, help="per-march setup, in march steps")
    args = ap.parse_args()
    import oracle
    import voxmap_amd as vx
    from voxmap_amd import presets, scenes
    cfg = presets.CONFIGS[args.config]
    grid = presets.scene_grid(cfg["scene"])
    field = vx.field_build(grid)
    noise = scenes.real_noise()
    W, H = cfg["w"], cfg["h"]
    up = 3.0 if cfg["scene"] == "s_up3" else 1.0
    fr = presets.camera_frame(cfg["camera"], W, H, scale=up, flags=vx.FLAG_FULL_QUALITY, shadow_samples=args.samples,
                              sun_radius=0.03 if args.samples > 1 else 0.0)
    o = oracle.Oracle(field, noise, exit=True)
    o.hold_exit_table(fr.params)
    L = oracle.lib()
    L.vxo_march_lengths.argtypes = [C.POINTER(oracle.OScene), C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int,
                                    C.c_int, C.c_int, C.c_void_p, C.c_int]
    L.vxo_march_lengths.restype = None
    rng = np.random.default_rng(7)
    maxrec = 2 * max(args.samples, 1) + 2
    tot = {"lockstep": 0.0, "ideal": 0.0}
    for t in (4, 8, 16, 32):
        tot[f"refill_T{t}"] = 0.0
    n = 0
    for _ in range(args.tiles):
        px0 = int(rng.integers(0, W // 8)) * 8
        py0 = int(rng.integers(0, H // 8)) * 8
        buf = np.empty((64, maxrec), np.int32)
        L.vxo_march_lengths(C.byref(o.sc), C.addressof(fr.params), W, H, px0, py0, 8, 8, buf.ctypes.data, maxrec)
        if not (buf >= 0).any():
            continue
        m = buf >= 0
        lit = (buf >> 16) & 1
        buf = np.where(m, buf & 0xFFFF, -1)
        tot.setdefault("fetch_lit", 0); tot.setdefault("fetch_unlit", 0)
        tot.setdefault("n_lit", 0); tot.setdefault("n_unlit", 0)
        tot["fetch_lit"] += int(buf[m & (lit == 1)].sum()); tot["fetch_unlit"] += int(buf[m & (lit == 0)].sum())
        tot["n_lit"] += int((m & (lit == 1)).sum()); tot["n_unlit"] += int((m & (lit == 0)).sum())
        n += 1
        tot["lockstep"] += lockstep(buf, args.setup)
        tot["ideal"] += buf[buf >= 0].sum() / 64.0
        for t in (4, 8, 16, 32):
            tot[f"refill_T{t}"] += refill(buf, args.setup, t)
        if args.samples > 1:
            tot["sorted_pool16"] = tot.get("sorted_pool16", 0.0) + sorted_pool(buf, args.setup, 16, 2 * args.setup)
    if args.samples > 1:
        # 32x8 blocks: lockstep vs the block-level two-class regroup
        bl = {"lockstep": 0.0, "classes": 0.0, "ideal": 0.0}
        nb = 0
        for _ in range(args.tiles // 4):
            px0 = int(rng.integers(0, W // 32)) * 32
            py0 = int(rng.integers(0, H // 8)) * 8
            buf = np.empty((8, 32, maxrec), np.int32)
            L.vxo_march_lengths(C.byref(o.sc), C.addressof(fr.params), W, H, px0, py0, 32, 8, buf.ctypes.data,
                                maxrec)
            # lanes of wave w: columns 8w .. 8w+7 of the block's 8 rows
            waves = np.concatenate([buf[:, 8 * w:8 * w + 8].reshape(64, maxrec) for w in range(4)])
            m = waves >= 0
            if not m.any():
                continue
            waves = np.where(m, waves & 0xFFFF, -1)
            nb += 1
            bl["lockstep"] += sum(lockstep(waves[64 * w:64 * (w + 1)], args.setup) for w in range(4))
            bl["classes"] += block_classes(waves, args.setup, 2 * args.setup)
            bl["ideal"] += waves[waves >= 0].sum() / 64.0
        for k, v in bl.items():
            print(f"  block {k:10s} {v / max(nb, 1):9.1f} wave steps per block ({v / bl['lockstep']:.3f} of lockstep)")
        # a global queue: every march of the sampled blocks after each fragment's
        # sample 0 (marched in place, lockstep per wave), sorted by that sample's
        # length, dealt 64 at a time (the best case for a grid-wide work queue)
        gl = {"lockstep": 0.0, "queue_sorted": 0.0, "queue_unsorted": 0.0, "queue_oracle_sorted": 0.0}
        rest, s0 = [], 0.0
        rng2 = np.random.default_rng(3)
        for _ in range(args.tiles // 4):
            px0 = int(rng2.integers(0, W // 32)) * 32
            py0 = int(rng2.integers(0, H // 8)) * 8
            buf = np.empty((8, 32, maxrec), np.int32)
            L.vxo_march_lengths(C.byref(o.sc), C.addressof(fr.params), W, H, px0, py0, 32, 8, buf.ctypes.data,
                                maxrec)
            waves = np.concatenate([buf[:, 8 * w:8 * w + 8].reshape(64, maxrec) for w in range(4)])
            m = waves >= 0
            if not m.any():
                continue
            waves = np.where(m, waves & 0xFFFF, -1)
            gl["lockstep"] += sum(lockstep(waves[64 * w:64 * (w + 1)], args.setup) for w in range(4))
            for w in range(4):
                col = waves[64 * w:64 * (w + 1), 0]
                if (col >= 0).any():
                    s0 += col.max() + args.setup
            for r in waves:
                if r[0] >= 0:
                    rest += [(int(r[0]), int(v)) for v in r[1:] if v >= 0]
        for name, order in (("queue_sorted", sorted(rest, key=lambda kv: -kv[0])), ("queue_unsorted", rest),
                            ("queue_oracle_sorted", sorted(rest, key=lambda kv: -kv[1]))):
            c = s0
            for i in range(0, len(order), 64):
                c += max(v for _, v in order[i:i + 64]) + 2 * args.setup
            gl[name] = c
        for k, v in gl.items():
            print(f"  global {k:14s} {v / max(nb, 1):9.1f} wave steps per block ({v / gl['lockstep']:.3f} of lockstep)")
    print(f"{args.config} samples={args.samples} tiles with marches={n} setup={args.setup} steps")
    for k in ("fetch_lit", "fetch_unlit", "n_lit", "n_unlit"):
        print(f"  {k:12s} {tot.pop(k, 0)}")
    for k, v in tot.items():
        print(f"  {k:12s} {v / max(n, 1):9.1f} wave steps per wave  ({v / tot['lockstep']:.3f} of lockstep)")


if __name__ == "__main__":
    main()
