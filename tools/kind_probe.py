"""Dev tool (build with EXTRA=-DIGX_KIND_PROBE, run with IGX_LIB_PATH on that
library): how often a k_extend wave shades specular and non-specular hits
together, per option set.  usage: kind_probe.py scene.json '<json list of option dicts>'"""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ignis-masterthesis_amd"))
import ignis_amd

scene = ignis_amd.Scene.from_file(os.path.join(ROOT, sys.argv[1]))
W, H = scene.film_size
dev = ignis_amd.Device(0)
dev.upload(scene)
p = ignis_amd.RenderParams(); p.width, p.height, p.spi = W, H, 8
for o in json.loads(sys.argv[2]) if len(sys.argv) > 2 else [{}]:
    for k, v in o.items():
        dev.set_option(k, v)
    dev.render(p); dev.synchronize()
    dev.reset_stats(); dev.set_option("instrument", 1); dev.clear()
    dev.render(p); dev.synchronize()
    s = dev.stats()
    dev.set_option("instrument", 0)
    waves, mixed, minority, mixed_b = (s["extend_cycles_" + k] for k in ("load", "trace", "shade", "store"))
    print(json.dumps({"opt": o, "waves": waves, "mixed_frac": round(mixed / max(1, waves), 4),
                      "mixed_b_frac_of_mixed": round(mixed_b / max(1, mixed), 4),
                      "minority_lanes_per_mixed_wave": round(minority / max(1, mixed), 2),
                      "extend_rays": s["extend_rays"]}), flush=True)
