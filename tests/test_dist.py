"""Screen-space sharding (voxmap_amd/dist.py) across ranks on CPU with gloo:
tile deal, padding to equal gather sizes, gather to rank 0, de-tile.  The tile
renderer is a CPU stand-in (the oracle frame cut into tiles) — on GPUs the same
ShardedFrame drives vx_render_tiles / vx_detile over RCCL (bench.py)."""
import os
import socket

import numpy as np
import pytest


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _frame():
    import oracle
    import voxmap_amd as vx
    from voxmap_amd import scenes
    g = scenes.small_proc(9, dims=(64, 40, 12), n_boxes=10, n_glass=2)
    field = vx.field_build(g)
    noise = np.full((16, 16, 4), 100, np.uint8)
    fr = vx.make_frame((32.0, 20.0, 14.0), (1.0, 0.0, 0.4), 100, 70)
    img, _ = oracle.Oracle(field, noise).render(fr.params, 100, 70)
    return img


def _worker(rank, world, port, ts, q, inflight=1, rounds=1):
    import torch
    import torch.distributed as dist

    from voxmap_amd.dist import ShardedFrame, TileLayout, detile_host
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        base = _frame()
        layout = TileLayout(100, 70, ts)

        def context(img):
            padded = np.zeros((layout.tiles_y * ts, layout.tiles_x * ts, 4), np.float32)
            padded[:70, :100] = img

            def render_tiles(ids, buf):
                for k, t in enumerate(ids):
                    x0, y0 = (t % layout.tiles_x) * ts, (t // layout.tiles_x) * ts
                    buf[k] = torch.from_numpy(padded[y0:y0 + ts, x0:x0 + ts])

            def detile(ids, cat, frame):
                frame.copy_(torch.from_numpy(detile_host(cat.numpy(), layout, ids)))

            return ShardedFrame(dist, layout, 4, torch.float32, "cpu", render_tiles, detile)

        # frames in flight (bench.py --inflight): one ShardedFrame per in-flight
        # frame, each with its own buffers and content, stepped alternately
        imgs = [base + np.float32(j) for j in range(inflight)]
        ctxs = [context(im) for im in imgs]
        ok = True
        for i in range(rounds * inflight):
            j = i % inflight
            out = ctxs[j].step()
            if rank == 0:
                ok &= bool(np.array_equal(out.numpy().view(np.uint32), imgs[j].view(np.uint32)))
        if rank == 0:
            q.put(ok)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,ts", [(2, 16), (3, 32), (5, 64)])
def test_sharded_frame_gloo(built, world, ts):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, ts, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=180)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert q.get(timeout=5) is True


def test_sharded_frames_in_flight_gloo(built):
    """Two frames in flight (bench.py's double buffering for N > 1): two
    ShardedFrames stepped alternately keep their own tiles and frames."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    world = 2
    procs = [ctx.Process(target=_worker, args=(r, world, port, 16, q, 2, 3)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=180)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert q.get(timeout=5) is True


def test_tile_layout_deal_is_a_partition():
    from voxmap_amd.dist import TileLayout
    lay = TileLayout(3840, 2160, 64)
    assert lay.n_tiles == 60 * 34
    for world in (1, 2, 4, 8, 7):
        lists = [lay.rank_tiles(world, r) for r in range(world)]
        flat = sorted(t for l in lists for t in l)
        assert flat == list(range(lay.n_tiles))
        padded, concat, per = lay.padded(world)
        assert all(len(l) == per for l in padded) and len(concat) == per * world
    tiny = TileLayout(10, 10, 16)
    padded, concat, per = tiny.padded(4)        # more ranks than tiles
    assert per == 1 and concat == [0, 0, 0, 0]
