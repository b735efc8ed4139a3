"""Dev tool: strong-scaling efficiency of the N-GPU tile-sharded bench,
simulated on one GPU: every rank's tile set (tile_offset = rank, tile_stride
= N) is rendered in turn as a full 256-spp frame; the job time at N is the
slowest rank's.  usage: shard_sim.py [scene] [tile sizes, comma-separated]"""
import json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ignis-masterthesis_amd"))
import ignis_amd

scene = ignis_amd.Scene.from_file(os.path.join(ROOT, sys.argv[1] if len(sys.argv) > 1 else "scenes/diamond_scene.json"))
from ignis_amd import shard
tiles = [int(t) for t in (sys.argv[2] if len(sys.argv) > 2 else "0").split(",")]
W, H = (int(v) for v in sys.argv[3].split("x")) if len(sys.argv) > 3 else scene.film_size
ITERS = int(sys.argv[4]) if len(sys.argv) > 4 else 32
dev = ignis_amd.Device(0)
dev.upload(scene)


def frame(n, rank, tile):
    dev.clear()
    p = ignis_amd.RenderParams()
    p.width, p.height, p.spi, p.iteration = W, H, 8, 0
    if n > 1:
        p.tile_size, p.tile_offset, p.tile_stride = tile or shard.balanced_tile(W, n), rank, n
    dev.render_iterations(p, ITERS)
    dev.synchronize()
    best = None
    for _ in range(2):
        dev.clear()
        t = time.perf_counter()
        dev.render_iterations(p, ITERS)
        dev.synchronize()
        dt = time.perf_counter() - t
        best = dt if best is None else min(best, dt)
    return best


t1 = frame(1, 0, 0)
print(json.dumps({"film": [W, H], "iterations": ITERS, "n": 1, "ms_frame": round(t1 * 1e3, 2)}), flush=True)
for tile in tiles:
    for n in (2, 4, 8):
        ts = [frame(n, r, tile) for r in range(n)]
        print(json.dumps({"tile": tile or shard.balanced_tile(W, n), "n": n, "ms_max_rank": round(max(ts) * 1e3, 2), "ms_min_rank": round(min(ts) * 1e3, 2),
                          "efficiency": round(t1 / (n * max(ts)), 3)}), flush=True)
