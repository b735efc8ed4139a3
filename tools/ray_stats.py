"""Dev tool: instrumented per-ray traversal statistics of one iteration
(node / instance / triangle visits per closest-hit and shadow ray, wave-level
node-loop and leaf-phase iterations per 64 rays, SIMD efficiency).
usage: ray_stats.py [scene.json] [options json]"""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ignis-masterthesis_amd"))
import ignis_amd

scene = ignis_amd.Scene.from_file(os.path.join(ROOT, sys.argv[1] if len(sys.argv) > 1 else "scenes/diamond_scene.json"))
W, H = scene.film_size
dev = ignis_amd.Device(0)
for k, v in (json.loads(sys.argv[2]) if len(sys.argv) > 2 else {}).items():
    dev.set_option(k, v)
dev.upload(scene)
p = ignis_amd.RenderParams(); p.width, p.height, p.spi = W, H, 8
dev.render(p); dev.synchronize()
dev.reset_stats(); dev.set_option("instrument", 1); dev.clear()
dev.render(p); dev.synchronize()
s = dev.stats()
n = s["camera_rays"] + s["bounce_rays"]
ns = max(1, s["shadow_rays"])
out = {"rays": n, "shadow_rays": s["shadow_rays"],
       "nodes/ray": s["node_visits"] / n, "inst/ray": s["leaf_visits"] / n, "tris/ray": s["tri_tests"] / n,
       "blas/ray": s["blas_enters"] / n,
       "wave_node_iters/64rays": 64 * s["wave_node_iters"] / n, "wave_leaf_iters/64rays": 64 * s["wave_leaf_iters"] / n,
       "simd_eff_nodes": s["node_visits"] / max(1, 64 * s["wave_node_iters"]),
       "sh_nodes/ray": s["shadow_node_visits"] / ns, "sh_tris/ray": s["shadow_tri_tests"] / ns,
       "sh_wave_node_iters/64rays": 64 * s["shadow_wave_node_iters"] / ns,
       "sh_wave_leaf_iters/64rays": 64 * s["shadow_wave_leaf_iters"] / ns,
       "depth": s["bvh_depth"], "width": s["bvh_width"], "lds_scene_bytes": s["lds_scene_bytes"],
       "table_bytes": s["table_bytes"]}
cyc = [s["extend_cycles_" + k] for k in ("load", "trace", "shade", "store")]
if sum(cyc):  # share of k_extend's wave time per phase (instrumented build)
    out.update({"ext_phase_" + k: c / sum(cyc) for k, c in zip(("load", "trace", "shade", "store"), cyc)})
    out["ext_wave_cycles/64rays"] = 64 * sum(cyc) / max(1, s["extend_rays"])
cc, cg = list(s["extend_class_cycles"]), list(s["extend_class_groups"])
if sum(cc):  # k_extend wave time by the class of the group: camera, A, B, C (trace / shade share, cycles per group)
    for i, k in enumerate(("cam", "A", "B", "C")):
        out[f"ext_{k}_trace_share"] = cc[i] / sum(cc)
        out[f"ext_{k}_shade_share"] = cc[4 + i] / sum(cc)
        out[f"ext_{k}_groups"] = cg[i]
        out[f"ext_{k}_cyc_per_group"] = (cc[i] + cc[4 + i]) / max(1, cg[i])
        out[f"ext_{k}_wave_node_iters_per_group"] = s["extend_class_node_iters"][i] / max(1, cg[i])
        out[f"ext_{k}_simd_eff"] = s["extend_class_node_visits"][i] / max(1, 64 * s["extend_class_node_iters"][i])
sc = list(s["extend_class_shade_cycles"])
if sum(sc):  # shading sub-phases per class: surface + material, emission, NEE, rest (share of the class's shade cycles)
    for i, k in enumerate(("cam", "A", "B", "C")):
        tot = max(1, sum(sc[4 * i:4 * i + 4]))
        out[f"ext_{k}_shade_split"] = [round(v / tot, 3) for v in sc[4 * i:4 * i + 4]]
        out[f"ext_{k}_shade_cyc_per_group"] = tot / max(1, cg[i])
g, it, vi, cy, oc = (list(s["shadow_class_" + k]) for k in ("groups", "node_iters", "node_visits", "cycles", "occluded"))
if sum(g):  # k_shadow by the shadow stream class of a group (A / B): share of wave time, cycles per group, occlusion
    for i, k in enumerate(("A", "B")):
        out[f"sh_{k}_groups"] = g[i]
        out[f"sh_{k}_cycle_share"] = cy[i] / max(1, sum(cy))
        out[f"sh_{k}_cyc_per_group"] = cy[i] / max(1, g[i])
        out[f"sh_{k}_wave_node_iters_per_group"] = it[i] / max(1, g[i])
        out[f"sh_{k}_simd_eff"] = vi[i] / max(1, 64 * it[i])
        out[f"sh_{k}_occluded_per_group"] = oc[i] / max(1, g[i])
if s["node_visits"]:  # closest-hit node visits in the TLAS and at hot-order ranks < 256 / 512 / 1280
    out["tlas_node_share"] = s["tlas_node_visits"] / s["node_visits"]
    for k, r in enumerate((256, 512, 1280)):
        out[f"node_rank_lt_{r}_share"] = s["hot_node_visits"][k] / s["node_visits"]
print(json.dumps({k: round(v, 3) if isinstance(v, float) else v for k, v in out.items()}))
