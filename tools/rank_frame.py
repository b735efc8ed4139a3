"""Dev tool: frame time of one rank's tile set (N-GPU bench shard, simulated
on one GPU) under several device-option sets.
usage: rank_frame.py scene N '<json list of option dicts>'"""
import json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ignis-masterthesis_amd"))
import ignis_amd
from ignis_amd import shard

scene = ignis_amd.Scene.from_file(os.path.join(ROOT, sys.argv[1]))
n = int(sys.argv[2])
opts = json.loads(sys.argv[3]) if len(sys.argv) > 3 else [{}]
W, H = scene.film_size
dev = ignis_amd.Device(0)
dev.upload(scene)
p = ignis_amd.RenderParams()
p.width, p.height, p.spi = W, H, 8
if n > 1:
    p.tile_size, p.tile_offset, p.tile_stride = shard.balanced_tile(W, n), 0, n
for o in opts:
    for k, v in o.items():
        dev.set_option(k, v)
    ts = []
    for rep in range(4):
        dev.clear()
        dev.reset_stats()
        dev.set_option("timing", 1 if rep == 3 else 0)
        t = time.perf_counter()
        dev.render_iterations(p, 32)
        dev.synchronize()
        ts.append(time.perf_counter() - t)
    st = dev.stats()
    dev.set_option("timing", 0)
    print(json.dumps({"opt": o, "n": n, "ms_frame": round(min(ts[1:3]) * 1e3, 2), "ms_timed": round(ts[3] * 1e3, 2),
                      "ext": round(st["ms_extend"], 2), "tr": round(st["ms_trace"], 2), "sh": round(st["ms_shadow"], 2),
                      "fin": round(st["ms_finish"], 2), "gen": round(st["ms_generate"], 2), "res": round(st["ms_resolve"], 2),
                      "wf_bounces": st["launches_extend"], "tail_rays": st["tail_bounce_rays"] + st["tail_shadow_rays"]}), flush=True)
