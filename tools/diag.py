"""Dev tool: instrumented pass over one iteration -- visits per ray and SIMD
efficiency (active lanes per wave-level loop iteration) of the traversal."""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ignis-masterthesis_amd"))
import ignis_amd

scene = ignis_amd.Scene.from_file(sys.argv[1] if len(sys.argv) > 1 and os.path.isabs(sys.argv[1]) else os.path.join(ROOT, sys.argv[1] if len(sys.argv) > 1 else "scenes/diamond_scene.json"))
W, H = scene.film_size
dev = ignis_amd.Device(0)
dev.upload(scene)
opts = json.loads(sys.argv[2]) if len(sys.argv) > 2 else {}
for k, v in opts.items():
    dev.set_option(k, v)
p = ignis_amd.RenderParams(); p.width, p.height, p.spi = W, H, 8
dev.render(p)
dev.reset_stats(); dev.set_option("instrument", 1)
p.iteration = 1; dev.render(p)
s = dev.stats()
rays = s["camera_rays"] + s["bounce_rays"]
out = {k: s[k] for k in ("camera_rays", "bounce_rays", "shadow_rays", "node_visits", "leaf_visits", "tri_tests", "blas_enters",
                          "wave_node_iters", "wave_leaf_iters", "shadow_node_visits", "shadow_wave_node_iters", "bvh_depth")}
out["nodes_per_ray"] = s["node_visits"] / rays
out["inst_per_ray"] = s["leaf_visits"] / rays
out["tris_per_ray"] = s["tri_tests"] / rays
out["simd_eff_nodes"] = s["node_visits"] / max(1, 64 * s["wave_node_iters"])
out["simd_eff_leaf_phase"] = (s["leaf_visits"] + s["tri_tests"]) / max(1, 64 * s["wave_leaf_iters"])
out["shadow_simd_eff_nodes"] = s["shadow_node_visits"] / max(1, 64 * s["shadow_wave_node_iters"])
print(json.dumps(out, indent=1))
