"""Dev tool: one rank's share of a tile-sharded frame (tile_offset 0 of N)
under several device-option sets (applied cumulatively, as sweep_frame.py), with the per-kernel times and the chunk
layout, to see where a rank's frame time goes.
usage: chunk_probe.py scene.json N '<json list of option dicts>' [iterations] [film size]"""
import json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ignis-masterthesis_amd"))
import ignis_amd
from ignis_amd import shard

scene = ignis_amd.Scene.from_file(os.path.join(ROOT, sys.argv[1]))
n = int(sys.argv[2])
opts = json.loads(sys.argv[3]) if len(sys.argv) > 3 else [{}]
iters = int(sys.argv[4]) if len(sys.argv) > 4 else 8
W = H = int(sys.argv[5]) if len(sys.argv) > 5 else 4096
dev = ignis_amd.Device(0)
dev.upload(scene)
p = ignis_amd.RenderParams()
p.width, p.height, p.spi = W, H, 8
if n > 1:
    p.tile_size, p.tile_offset, p.tile_stride = shard.balanced_tile(W, n), 0, n
for o in opts:
    for k, v in o.items():
        dev.set_option(k, v)
    dev.clear()
    dev.render_iterations(p, iters)
    dev.synchronize()
    best = None
    for rep in range(2):
        dev.reset_stats()
        dev.set_option("timing", 1)
        dev.clear()
        t = time.perf_counter()
        dev.render_iterations(p, iters)
        dev.synchronize()
        dt = time.perf_counter() - t
        s = dev.stats()
        dev.set_option("timing", 0)
        if best is None or dt < best[0]:
            best = (dt, s)
    dt, s = best
    rays = s["camera_rays"] + s["bounce_rays"] + s["shadow_rays"]
    print(json.dumps({"n": n, "opt": o, "ms_frame": round(dt * 1e3, 2), "Mrays/s": round(rays / dt / 1e6, 1),
                      "ns_per_camera_ray": round(dt * 1e9 / max(1, s["camera_rays"]), 3),
                      "ext": round(s["ms_extend"], 2), "sh": round(s["ms_shadow"], 2), "fin": round(s["ms_finish"], 2),
                      "gen": round(s["ms_generate"], 2), "res": round(s["ms_resolve"], 2),
                      "launches_ext": s["launches_extend"], "tail_rays": s["tail_bounce_rays"] + s["tail_shadow_rays"],
                      "slot_bytes": s["slot_bytes"]}), flush=True)
dev.close()
