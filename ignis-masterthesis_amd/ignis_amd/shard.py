"""Tile sharding of the film across ranks.

The film is cut into T×T tiles, numbered row-major; tile t belongs to rank
t % N (round-robin, for load balance).  Each rank renders only its tiles
(igx_render_params.tile_offset = rank, tile_stride = N) and `igx_pack_tiles`
packs them as [tile k of this rank][row][col][rgb], padded to T×T.  After an
all_gather of equal-size packed buffers every rank assembles the frame with
one scatter through the destination table built here.
"""
import math

import numpy as np


def balanced_tile(width, n_ranks, lo=32, hi=64, prefer=40):
    """Tile size for n_ranks: the one nearest `prefer` in [lo, hi] whose tile
    column count is coprime with n_ranks, so round-robin ownership (t % N)
    staggers from row to row instead of giving each rank whole tile columns.
    Whole columns load ranks unevenly when the image content is uneven
    (diamond, 8 ranks, 64-px tiles: slowest rank 28.3 ms, fastest 22.6 ms;
    40-px tiles, 25 columns: 25.0 / 24.5 ms; tools/shard_sim.py)."""
    for t in sorted(range(lo, hi + 1), key=lambda t: (abs(t - prefer), t)):
        if math.gcd((width + t - 1) // t, max(1, n_ranks)) == 1:
            return t
    return prefer


def tile_grid(width, height, tile):
    return (width + tile - 1) // tile, (height + tile - 1) // tile


def owned_tiles(width, height, tile, rank, n_ranks):
    tx, ty = tile_grid(width, height, tile)
    return np.arange(rank, tx * ty, n_ranks)


def max_tiles_per_rank(width, height, tile, n_ranks):
    tx, ty = tile_grid(width, height, tile)
    return (tx * ty + n_ranks - 1) // n_ranks


def packed_destinations(width, height, tile, n_ranks):
    """For the concatenation of every rank's packed buffer (each padded to
    max_tiles_per_rank tiles), the destination pixel index in the width×height
    film, or -1 for padding and for tile pixels outside the film."""
    tx, _ = tile_grid(width, height, tile)
    per_rank = max_tiles_per_rank(width, height, tile, n_ranks) * tile * tile
    yy, xx = np.mgrid[0:tile, 0:tile]
    out = []
    for r in range(n_ranks):
        t = owned_tiles(width, height, tile, r, n_ranks)
        gy = (t // tx)[:, None, None] * tile + yy
        gx = (t % tx)[:, None, None] * tile + xx
        pix = np.where((gx < width) & (gy < height), gy * width + gx, -1).reshape(-1)
        full = np.full(per_rank, -1, np.int64)
        full[: pix.size] = pix
        out.append(full)
    return np.concatenate(out)


def assemble(gathered_rgb, dst, frame_rgb):
    """Scatter the gathered packed pixels ((R*P, 3) rows, torch or numpy) into
    frame_rgb ((W*H, 3)) through the table from packed_destinations."""
    valid = dst >= 0
    frame_rgb[dst[valid]] = gathered_rgb[valid]
    return frame_rgb


def rank_summary(dist, values, device="cpu"):
    """Per-rank figures of a sharded frame, collected on every rank: for each
    key of `values` (this rank's float) the per-rank list in rank order, its
    min, max and mean.  `dist` is torch.distributed (world > 1) or None (one
    rank); the all_gather runs on `device` ("cuda" over RCCL, "cpu" over
    gloo).  bench.py reports the frame, pack and gather times this way, so a
    sub-linear scaling curve shows whether a slow rank or the gather costs it."""
    import torch

    keys = sorted(values)
    mine = torch.tensor([float(values[k]) for k in keys], dtype=torch.float64, device=device)
    if dist is not None and dist.get_world_size() > 1:
        parts = [torch.zeros_like(mine) for _ in range(dist.get_world_size())]
        dist.all_gather(parts, mine)
        table = torch.stack(parts).cpu().numpy()
    else:
        table = mine.cpu().numpy()[None, :]
    out = {}
    for j, k in enumerate(keys):
        col = [round(float(v), 3) for v in table[:, j]]
        out[k] = {"min": min(col), "max": max(col), "mean": round(float(np.mean(col)), 3), "per_rank": col}
    return out
