"""Dev tool: time one diamond iteration under different device options."""
import json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ignis-masterthesis_amd"))
import ignis_amd

scene = ignis_amd.Scene.from_file(os.path.join(ROOT, sys.argv[1] if len(sys.argv) > 1 else "scenes/diamond_scene.json"))
W, H = scene.film_size
dev = ignis_amd.Device(0)
dev.upload(scene)
opts = json.loads(sys.argv[2]) if len(sys.argv) > 2 else [{}]
p = ignis_amd.RenderParams(); p.width, p.height, p.spi = W, H, 8
for o in opts:
    for k, v in o.items():
        dev.set_option(k, v)
    if any(k in ("bvh_width", "bvh_leaf_size") for k in o):
        dev.upload(scene)  # these take effect at upload
    for it in range(2):
        p.iteration = it; dev.render(p)
    dev.reset_stats(); dev.set_option("timing", 1)
    t = time.perf_counter(); K = 6
    for it in range(K):
        p.iteration = 10 + it; dev.render(p)
    dev.synchronize()
    dt = (time.perf_counter() - t) / K
    s = dev.stats(); dev.set_option("timing", 0)
    rays = (s["camera_rays"] + s["bounce_rays"] + s["shadow_rays"]) / K
    print(json.dumps({"opt": o, "ms_iter": round(dt * 1e3, 3), "Mrays/s": round(rays / dt / 1e6, 1),
                      "tr": round(s["ms_trace"] / K, 3), "ext": round(s["ms_extend"] / K, 3), "sh": round(s["ms_shadow"] / K, 3), "fin": round(s["ms_finish"] / K, 3),
                      "gen": round(s["ms_generate"] / K, 3), "res": round(s["ms_resolve"] / K, 3),
                      "wf_bounces": s["launches_extend"] / K, "tail_rays": (s["tail_bounce_rays"] + s["tail_shadow_rays"]) / K,
                      "depth": s["bvh_depth"], "width": s["bvh_width"]}), flush=True)
