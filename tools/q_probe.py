"""Dev tool: quantised 4-wide nodes against the 128-B nodes on one scene --
closest hits of camera and random rays (which rays differ, and whether the
quantised tree found a nearer hit = a triangle the exact boxes skipped, or a
farther one = a triangle it missed) and an image comparison.
usage: q_probe.py scene.json"""
import json, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ignis-masterthesis_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)
import ignis_amd
from test_gpu import camera_rays, random_rays

sc = ignis_amd.Scene.from_file(os.path.join(ROOT, sys.argv[1]))
dev = ignis_amd.Device(0)
rays = np.concatenate([camera_rays(sc, 400, 400, jitter=0.37), random_rays(sc, 400000, seed=11)])
res, imgs = [], []
for q in (0, 1):
    dev.set_option("bvh_quantize", q)
    dev.upload(sc)
    res.append(dev.trace_hits(rays, 0x1))
    p = ignis_amd.RenderParams()
    p.width, p.height, p.spi = 256, 256, 4
    dev.clear()
    dev.render(p)
    imgs.append(dev.framebuffer(256 * 256 * 3)[0])
(e0, t0), (e1, t1) = res
diff = np.any(e0 != e1, axis=1) | (t0[:, 0] != t1[:, 0])
idx = np.nonzero(diff)[0]
nearer = int(np.sum(t1[idx, 0] < t0[idx, 0]))
farther = int(np.sum(t1[idx, 0] > t0[idx, 0]))
im = np.abs(imgs[0] - imgs[1]) > 0
out = {"rays": int(len(rays)), "differ": int(len(idx)), "quantised_nearer": nearer, "quantised_farther": farther,
       "equal_t_other_prim": int(len(idx) - nearer - farther),
       "image_px_differ": int(im.reshape(-1, 3).any(axis=1).sum()), "max_rel_t": float(np.max(np.abs(t1[idx, 0] - t0[idx, 0]) / np.maximum(np.abs(t0[idx, 0]), 1e-30))) if len(idx) else 0.0,
       "examples": [[rays[i].tolist(), e0[i].tolist(), t0[i].tolist(), e1[i].tolist(), t1[i].tolist()] for i in idx[:3]]}
print(json.dumps(out))
