"""Tile sharding and the frame gather on CPU: the destination
table, and a world-size-2 gloo all_gather + assemble, mirroring bench.py's
multi-GPU path (which runs the same code over RCCL)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from ignis_amd import shard


def pack_host(frame_rgb, width, height, tile, rank, n_ranks):
    """Host restatement of k_pack_tiles' layout: owned tiles in ascending order,
    each T×T row-major, pixels outside the film zero, padded to the max tile count."""
    out = np.zeros((shard.max_tiles_per_rank(width, height, tile, n_ranks), tile, tile, 3), np.float32)
    tx, _ = shard.tile_grid(width, height, tile)
    img = frame_rgb.reshape(height, width, 3)
    for k, t in enumerate(shard.owned_tiles(width, height, tile, rank, n_ranks)):
        y0, x0 = (t // tx) * tile, (t % tx) * tile
        blk = img[y0:y0 + tile, x0:x0 + tile]
        out[k, : blk.shape[0], : blk.shape[1]] = blk
    return out.reshape(-1)


@pytest.mark.parametrize("w,h,T,N", [(200, 150, 64, 3), (1000, 1000, 64, 8), (64, 64, 64, 2), (130, 70, 16, 5)])
def test_destinations_cover_film_once(w, h, T, N):
    dst = shard.packed_destinations(w, h, T, N)
    v = dst[dst >= 0]
    assert v.size == w * h
    assert np.array_equal(np.sort(v), np.arange(w * h))


@pytest.mark.parametrize("w,h,T,N", [(200, 150, 64, 3), (130, 70, 16, 5)])
def test_pack_assemble_roundtrip(w, h, T, N):
    rng = np.random.default_rng(1)
    frame = rng.random((w * h, 3), dtype=np.float32)
    packs = np.concatenate([pack_host(frame, w, h, T, r, N) for r in range(N)])
    out = shard.assemble(packs.reshape(-1, 3), shard.packed_destinations(w, h, T, N), np.zeros_like(frame))
    np.testing.assert_array_equal(out, frame)


@pytest.mark.parametrize("w,N", [(1000, 2), (1000, 4), (1000, 8), (4096, 8), (1000, 5), (1000, 3)])
def test_balanced_tile_staggers_ownership(w, N):
    """Tile column count coprime with N: along a tile row, consecutive rows start
    the round-robin at different ranks, so no rank owns whole tile columns."""
    import math
    T = shard.balanced_tile(w, N)
    tx, _ = shard.tile_grid(w, w, T)
    assert 32 <= T <= 64 and math.gcd(tx, N) == 1
    owners_col0 = {(r * tx) % N for r in range(N)}
    assert owners_col0 == set(range(N))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, w, h, T, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rng = np.random.default_rng(7)
    frame = rng.random((w * h, 3), dtype=np.float32)   # same "render" on every rank
    # each rank keeps only its tiles, as the device does under tile sharding
    pack = torch.from_numpy(pack_host(frame, w, h, T, rank, world))
    # gather to rank 0 only, as bench.py does it over RCCL
    bufs = [torch.zeros_like(pack) for _ in range(world)] if rank == 0 else None
    dist.gather(pack, bufs, dst=0)
    if rank == 0:
        dst = torch.from_numpy(shard.packed_destinations(w, h, T, world))
        out = shard.assemble(torch.cat(bufs).view(-1, 3), dst, torch.zeros((w * h, 3)))
        ok = bool(torch.equal(out, torch.from_numpy(frame)))
    else:
        ok = True
    # max-over-ranks timing reduction used by bench.py
    t = torch.tensor([float(rank + 1)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    q.put((rank, ok, float(t.item())))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_gather_assembles_frame():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    w, h, T, world = 200, 150, 64, 2
    # also exercised with world 3 below
    procs = [ctx.Process(target=_worker, args=(r, world, port, w, h, T, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(ok for _, ok, _ in res), res
    assert all(t == float(world) for _, _, t in res)


def test_gloo_world3_gather_assembles_frame():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    w, h, world = 4096 // 16, 4096 // 16, 3
    T = shard.balanced_tile(w, world)
    procs = [ctx.Process(target=_worker, args=(r, world, port, w, h, T, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(ok for _, ok, _ in res), res


def _summary_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    s = shard.rank_summary(dist, {"frame_ms": 10.0 * (rank + 1), "gather_ms": 0.5 + rank})
    q.put((rank, s))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_rank_summary():
    """bench.py's per-rank breakdown (frame / pack / gather ms at N > 1): every
    rank sees every rank's value, in rank order, with min / max / mean."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_summary_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=120) for _ in range(2)), key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for _, s in res:
        assert s["frame_ms"] == {"min": 10.0, "max": 20.0, "mean": 15.0, "per_rank": [10.0, 20.0]}
        assert s["gather_ms"]["per_rank"] == [0.5, 1.5]


def test_rank_summary_single_rank():
    s = shard.rank_summary(None, {"frame_ms": 3.25})
    assert s == {"frame_ms": {"min": 3.25, "max": 3.25, "mean": 3.25, "per_rank": [3.25]}}


def test_rank_stream_slots_by_share():
    """bench.py keeps one stream slot per device handle when a rank's share of
    a frame is one chunk (the diamond at any N), two when it spans several
    (config 5 at N = 2 / 4 / 8), so consecutive chunks of a frame overlap."""
    import importlib.util
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(root, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    from ignis_amd import shard
    for n in (2, 4, 8):
        assert bench.rank_stream_slots(1000, 1000, shard.balanced_tile(1000, n), n, 8, 32) == 1
        assert bench.rank_stream_slots(4096, 4096, shard.balanced_tile(4096, n), n, 8, 8) == 2
    # exactly one chunk: 2^27 paths
    assert bench.rank_stream_slots(4096, 4096, 4096, 1, 8, 1) == 1
    assert bench.rank_stream_slots(4096, 4096, 4096, 1, 8, 2) == 2


def _load_bench():
    import importlib.util
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(root, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    return bench


def _preflight_worker(rank, world, port, fail_rank, q):
    """bench.sharded_line with stand-ins for the device: rank `fail_rank`
    fails while rendering its pre-flight frame (as an out-of-memory render
    does); every rank must return the error line instead of entering the
    line's gathers and barriers."""
    import types
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    bench = _load_bench()

    class Dev:
        def clear(self):
            pass

        def render_iterations(self, p, n):
            if rank == fail_rank:
                raise RuntimeError("hipMalloc: out of memory")

        def synchronize(self):
            pass

    class Frames:
        def __init__(self, *a):
            self.devs = [Dev(), Dev()]

        def params(self, it=0):
            return None

        def measure(self, steps, warmup):
            raise AssertionError("measure reached after a failed pre-flight")

        def close(self):
            self.devs = []

    bench.RankFrames = Frames
    ig = types.SimpleNamespace(Scene=types.SimpleNamespace(from_file=lambda path: None))
    line = bench.sharded_line(ig, torch, dist, "s_deep.json", 64, 8, 64, rank, world, 0, "cpu", 1, True)
    q.put((rank, line))
    dist.barrier()  # the ranks still agree on the next collective
    dist.destroy_process_group()


def test_gloo_world2_config5_preflight_failure_does_not_hang():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_preflight_worker, args=(r, 2, port, 1, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[1]["error"].startswith("rank 1: RuntimeError")
    assert res[0]["error"] == "another rank failed its pre-flight frame"
