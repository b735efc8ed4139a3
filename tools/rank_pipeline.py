"""Dev tool: average frame time of one rank's tile set (N-GPU bench shard,
simulated on one GPU) over K back-to-back frames, with one device handle
(each frame drained before the next, as the gather requires) and with two
handles alternating (bench.py's N > 1 pipelining: frame k+1 queued before
frame k is drained).  usage: rank_pipeline.py scene N [K] [stream_slots] [iterations] [square film size]
IGX_PIPE_OPTS='{"option": value, ...}' sets device options on both handles; IGX_PIPE_THREADS=1 compares
two handles rendering sequentially with two handles whose frames render on worker threads."""
import json, os, sys, threading, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ignis-masterthesis_amd"))
import ignis_amd
from ignis_amd import shard

scene = ignis_amd.Scene.from_file(os.path.join(ROOT, sys.argv[1]))
n = int(sys.argv[2])
K = int(sys.argv[3]) if len(sys.argv) > 3 else 6
W, H = scene.film_size
ITERS = int(sys.argv[5]) if len(sys.argv) > 5 else 32
if len(sys.argv) > 6 and int(sys.argv[6]) > 0:
    W = H = int(sys.argv[6])
devs = [ignis_amd.Device(0), ignis_amd.Device(0)]
slots = int(sys.argv[4]) if len(sys.argv) > 4 else 2
extra = json.loads(os.environ.get("IGX_PIPE_OPTS", "{}"))
READY = os.environ.get("IGX_PIPE_READY") == "1"
for d in devs:
    d.upload(scene)
    d.set_option("stream_slots", slots)
    for k, v in extra.items():
        d.set_option(k, v)
p = ignis_amd.RenderParams()
p.width, p.height, p.spi = W, H, 8
if n > 1:
    p.tile_size, p.tile_offset, p.tile_stride = shard.balanced_tile(W, n), 0, n


def run(handles):
    pending = None
    t = time.perf_counter()
    for k in range(K):
        d = handles[k % len(handles)]
        d.clear()
        d.render_iterations(p, ITERS)
        if READY and len(handles) > 1:
            d.wait_ready()  # bench.py's N > 1 order: the next frame starts in this one's late bounces
        if pending is not None:
            pending.synchronize()
        pending = d
        if len(handles) == 1:
            d.synchronize()
            pending = None
    if pending is not None:
        pending.synchronize()
    return (time.perf_counter() - t) / K


def run_threads(handles):
    """two handles, each frame rendered on a worker thread (ctypes releases the
    GIL): frame k+1's bounces are queued while frame k's last bounces run"""
    inflight = None
    t = time.perf_counter()
    for k in range(K):
        d = handles[k % 2]
        th = threading.Thread(target=lambda d=d: (d.clear(), d.render_iterations(p, ITERS)))
        th.start()
        if inflight is not None:
            inflight[1].join()
            inflight[0].synchronize()
        inflight = (d, th)
    inflight[1].join()
    inflight[0].synchronize()
    return (time.perf_counter() - t) / K


if os.environ.get("IGX_PIPE_THREADS"):
    for _ in range(2):
        run(devs)
        print(json.dumps({"n": n, "stream_slots": slots, "opts": extra, "handles": 2, "threads": False,
                          "ms_per_frame": round(run(devs) * 1e3, 2)}), flush=True)
        run_threads(devs)
        print(json.dumps({"n": n, "stream_slots": slots, "opts": extra, "handles": 2, "threads": True,
                          "ms_per_frame": round(run_threads(devs) * 1e3, 2)}), flush=True)
    sys.exit(0)

for handles in (devs[:1], devs, devs[:1], devs):
    run(handles)
    print(json.dumps({"n": n, "stream_slots": slots, "opts": extra, "ready": READY, "handles": len(handles), "ms_per_frame": round(run(handles) * 1e3, 2),
                      "slot_gb_per_handle": [round(d.stats()["slot_bytes"] / 1e9, 2) for d in handles]}), flush=True)
