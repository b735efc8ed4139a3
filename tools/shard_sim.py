"""Dev tool: per-rank frame time of the N-GPU tile-sharded bench, simulated on
one GPU by rendering only rank 0's tiles (tile_offset 0, tile_stride N) --
the strong-scaling efficiency the driver's multi-GPU runs can reach."""
import json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ignis-masterthesis_amd"))
import ignis_amd

scene = ignis_amd.Scene.from_file(os.path.join(ROOT, sys.argv[1] if len(sys.argv) > 1 else "scenes/diamond_scene.json"))
W, H = scene.film_size
dev = ignis_amd.Device(0)
dev.upload(scene)
opts = json.loads(sys.argv[2]) if len(sys.argv) > 2 else {}
batched = opts.pop("batched", 1)
for k, v in opts.items():
    dev.set_option(k, v)
base = None
for n in (1, 2, 4, 8):
    def frame():
        dev.clear()
        p = ignis_amd.RenderParams()
        p.width, p.height, p.spi, p.iteration = W, H, 8, 0
        if n > 1:
            p.tile_size, p.tile_offset, p.tile_stride = 64, 0, n
        if batched:
            dev.render_iterations(p, 32)
        else:
            for it in range(32):
                p.iteration = it
                dev.render(p)
        dev.synchronize()
    frame()
    t = time.perf_counter()
    frame()
    dt = time.perf_counter() - t
    base = base or dt
    print(json.dumps({"batched": batched, "n": n, "ms_frame_rank0": round(dt * 1e3, 2), "efficiency": round(base / (n * dt), 3)}), flush=True)
