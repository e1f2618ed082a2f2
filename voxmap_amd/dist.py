"""Screen-space sharding of one frame across GPUs.

Pixels are independent (render.frag reads only the replicated field and noise
textures), so a frame is cut into square tiles dealt round-robin to ranks —
interleaving balances cheap sky tiles against expensive geometry tiles.  Each
rank renders its tiles into a compact tile-major buffer (vx_render_tiles);
rank 0 gathers the buffers with one collective (torch.distributed.gather, RCCL
over xGMI on MI355X nodes, gloo in CPU tests) and scatters them into the frame
(vx_detile).  There is no other exchange.

Gather sizes must match across ranks, so every rank's list is padded to the
longest one by repeating its last tile (the repeat re-writes identical pixels).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np


@dataclass(frozen=True)
class TileLayout:
    width: int
    height: int
    tile: int

    @property
    def tiles_x(self) -> int:
        return -(-self.width // self.tile)

    @property
    def tiles_y(self) -> int:
        return -(-self.height // self.tile)

    @property
    def n_tiles(self) -> int:
        return self.tiles_x * self.tiles_y

    def rank_tiles(self, world: int, rank: int) -> list:
        """Round-robin deal (tile t -> rank t % world)."""
        return list(range(rank, self.n_tiles, world))

    def padded(self, world: int):
        """(per-rank padded lists, their concatenation in rank order, tiles per rank)."""
        lists = [self.rank_tiles(world, r) for r in range(world)]
        per = max(len(l) for l in lists)
        if per == 0:
            raise ValueError("frame has no tiles")
        padded = []
        for l in lists:
            if not l:            # more ranks than tiles: repeat tile 0 (rewrites identical pixels)
                l = [0]
            padded.append(l + [l[-1]] * (per - len(l)))
        concat = [t for l in padded for t in l]
        return padded, concat, per


def detile_host(tiles: np.ndarray, layout: TileLayout, ids) -> np.ndarray:
    """Host twin of vx_detile for CPU checks: tiles (n, ts, ts, C) -> frame (h, w, C)."""
    ts = layout.tile
    frame = np.zeros((layout.height, layout.width, tiles.shape[-1]), tiles.dtype)
    for k, t in enumerate(ids):
        x0, y0 = (t % layout.tiles_x) * ts, (t // layout.tiles_x) * ts
        h = min(ts, layout.height - y0)
        w = min(ts, layout.width - x0)
        frame[y0:y0 + h, x0:x0 + w] = tiles[k, :h, :w]
    return frame


class ShardedFrame:
    """One rank's part of a sharded frame: render my tiles, gather to rank 0, de-tile.

    ``render_tiles(ids, out_tensor)`` and ``detile(concat_ids, tiles_tensor, frame_tensor)``
    are injected: on GPUs they are Scene.render_tiles / Scene.detile over device tensors;
    CPU tests pass host stand-ins.  ``dist`` is torch.distributed (initialised).
    """

    def __init__(self, dist, layout: TileLayout, channels: int, dtype, device, render_tiles, detile):
        import torch
        self.dist = dist
        self.layout = layout
        self.world = dist.get_world_size()
        self.rank = dist.get_rank()
        lists, self.concat, self.per = layout.padded(self.world)
        self.mine = lists[self.rank]
        ts = layout.tile
        self.buf = torch.empty((self.per, ts, ts, channels), dtype=dtype, device=device)
        if self.rank == 0:
            self.parts = [torch.empty_like(self.buf) for _ in range(self.world)]
            self.cat = torch.empty((self.world * self.per, ts, ts, channels), dtype=dtype, device=device)
            self.frame = torch.empty((layout.height, layout.width, channels), dtype=dtype, device=device)
        else:
            self.parts = self.cat = self.frame = None
        self._render = render_tiles
        self._detile = detile

    def step(self):
        import torch
        self._render(self.mine, self.buf)
        self.dist.gather(self.buf, gather_list=self.parts, dst=0)
        if self.rank == 0:
            torch.cat(self.parts, out=self.cat)
            self._detile(self.concat, self.cat, self.frame)
        return self.frame
