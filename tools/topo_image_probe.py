"""Dev probe: the same frame under two BVH builder settings; prints the BVH
shape of each and how many pixels differ (and by how much).
usage: topo_image_probe.py scene.json '{opts A}' '{opts B}' [spi]"""
import json, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ignis-masterthesis_amd"))
import ignis_amd

sc = ignis_amd.Scene.from_file(os.path.join(ROOT, sys.argv[1]))
W, H = sc.film_size
spi = int(sys.argv[4]) if len(sys.argv) > 4 else 8
dev = ignis_amd.Device(0)
imgs = []
for o in (json.loads(sys.argv[2]), json.loads(sys.argv[3])):
    for k, v in o.items():
        dev.set_option(k, v)
    dev.upload(sc)
    st = dev.stats()
    dev.clear(); dev.reset_stats()
    p = ignis_amd.RenderParams(); p.width, p.height, p.spi = W, H, spi
    dev.render(p)
    fb, _ = dev.framebuffer(W * H * 3)
    s2 = dev.stats()
    print(json.dumps({"opts": o, "bvh_width": st["bvh_width"], "bvh_depth": st["bvh_depth"],
                      "rays": [s2["camera_rays"], s2["bounce_rays"], s2["shadow_rays"]]}))
    imgs.append(fb.reshape(H, W, 3))
a, b = imgs
d = np.any(a != b, axis=2)
ys, xs = np.nonzero(d)
rel = np.abs(a - b).max(axis=2)[d] / np.maximum(np.abs(a).max(axis=2)[d], 1e-6) if d.any() else np.array([0.0])
print(json.dumps({"pixels_differ": int(d.sum()), "max_rel": float(rel.max()), "first": list(zip(ys[:5].tolist(), xs[:5].tolist()))}))
