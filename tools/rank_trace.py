"""Dev tool: workload for a kernel trace of one rank's frames at N > 1 (the
bench's order: two handles alternating, the next frame queued once the
current one is in its late bounces, igx_wait_ready): K warm-up frames, then K
measured ones.  usage: rank_trace.py scene N [K] [iterations] [square size] [stream_slots]"""
import json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ignis-masterthesis_amd"))
import ignis_amd
from ignis_amd import shard

scene = ignis_amd.Scene.from_file(os.path.join(ROOT, sys.argv[1]))
n = int(sys.argv[2])
K = int(sys.argv[3]) if len(sys.argv) > 3 else 6
ITERS = int(sys.argv[4]) if len(sys.argv) > 4 else 32
W, H = scene.film_size
if len(sys.argv) > 5 and int(sys.argv[5]) > 0:
    W = H = int(sys.argv[5])
slots = int(sys.argv[6]) if len(sys.argv) > 6 else 1
devs = [ignis_amd.Device(0), ignis_amd.Device(0)]
for d in devs:
    d.upload(scene)
    d.set_option("stream_slots", slots)
    for k, v in json.loads(os.environ.get("IGX_PIPE_OPTS", "{}")).items():
        d.set_option(k, v)
p = ignis_amd.RenderParams()
p.width, p.height, p.spi = W, H, 8
p.tile_size, p.tile_offset, p.tile_stride = shard.balanced_tile(W, n), 0, n


def frames(k_frames):
    pending = None
    t = time.perf_counter()
    for k in range(k_frames):
        d = devs[k % 2]
        d.clear()
        d.render_iterations(p, ITERS)
        d.wait_ready()
        if pending is not None:
            pending.synchronize()
        pending = d
    pending.synchronize()
    return (time.perf_counter() - t) / k_frames


frames(K)
print(json.dumps({"n": n, "frames": K, "ms_per_frame": round(frames(K) * 1e3, 2)}), flush=True)
