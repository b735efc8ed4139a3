"""Dev tool: one bench frame (all iterations in one igx_render_iterations call,
as bench.py renders them) of a scene under several device-option sets.
usage: sweep_frame.py scene.json '<json list of option dicts>' [iterations] [film WxH]"""
import json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ignis-masterthesis_amd"))
import ignis_amd

scene = ignis_amd.Scene.from_file(os.path.join(ROOT, sys.argv[1]))
W, H = (int(v) for v in sys.argv[4].split("x")) if len(sys.argv) > 4 else scene.film_size
opts = json.loads(sys.argv[2]) if len(sys.argv) > 2 else [{}]
iters = int(sys.argv[3]) if len(sys.argv) > 3 else 32
dev = ignis_amd.Device(0)
dev.upload(scene)
p = ignis_amd.RenderParams()
p.width, p.height, p.spi = W, H, 8
for o in opts:
    for k, v in o.items():
        dev.set_option(k, v)
    if any(k in ("bvh_width", "bvh_leaf_size", "spatial_splits", "sah_node_cost_pct", "rebuild_bvh", "enclosing", "bvh_bins", "face_normals", "face_shade", "bvh_quantize") for k in o):
        dev.upload(scene)
    dev.clear()
    dev.render_iterations(p, iters)  # warm-up, buffers sized
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
    import hashlib
    fb, _ = dev.framebuffer(W * H * 3)
    md5 = hashlib.md5(fb.tobytes()).hexdigest()[:12]
    print(json.dumps({"opt": o, "ms_frame": round(dt * 1e3, 2), "Mrays/s": round(rays / dt / 1e6, 1),
                      "ext": round(s["ms_extend"], 2), "tr": round(s["ms_trace"], 2), "sh": round(s["ms_shadow"], 2),
                      "fin": round(s["ms_finish"], 2), "gen": round(s["ms_generate"], 2), "res": round(s["ms_resolve"], 2), "tail_rays": s["tail_bounce_rays"] + s["tail_shadow_rays"],
                      "launches_ext": s["launches_extend"], "treelet": s.get("treelet_nodes"), "fb_md5": md5}), flush=True)
dev.close()
