"""Dev probe: closest hits of the same rays under two BVH builder settings
(device options applied before upload); prints how many rays differ and the
first few differences.  usage: topo_probe.py scene.json '{opts A}' '{opts B}' [n]"""
import json, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ignis-masterthesis_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)
import ignis_amd
from test_gpu import camera_rays, random_rays

sc = ignis_amd.Scene.from_file(os.path.join(ROOT, sys.argv[1]))
n = int(sys.argv[4]) if len(sys.argv) > 4 else 2_000_000
rays = np.concatenate([camera_rays(sc, 1000, 1000, jitter=0.37), random_rays(sc, n, seed=9)])
dev = ignis_amd.Device(0)
res = []
for o in (json.loads(sys.argv[2]), json.loads(sys.argv[3])):
    for k, v in o.items():
        dev.set_option(k, v)
    dev.upload(sc)
    res.append(dev.trace_hits(rays, 0x1))
# second generation: rays leaving the first hits in random directions (bounce-like)
ea0, ta0 = res[0]
hit = ea0[:, 0] >= 0
rng = np.random.default_rng(5)
sec = np.zeros((int(hit.sum()), 8), np.float32)
sec[:, 0:3] = rays[hit, 0:3] + rays[hit, 3:6] * ta0[hit, 0:1]
dd = rng.normal(size=(sec.shape[0], 3)); dd /= np.linalg.norm(dd, axis=1, keepdims=True)
sec[:, 3:6], sec[:, 6], sec[:, 7] = dd, 1e-3, 3.4e38
res2 = []
for o in (json.loads(sys.argv[2]), json.loads(sys.argv[3])):
    for k, v in o.items():
        dev.set_option(k, v)
    dev.upload(sc)
    res2.append(dev.trace_hits(sec, 0x4))
(sa, sta), (sb, stb) = res2
sdiff = np.flatnonzero(np.any(sa != sb, axis=1) | np.any(sta != stb, axis=1))
print(json.dumps({"secondary_rays": len(sec), "secondary_differ": int(sdiff.size)}))
for i in sdiff[:8]:
    print(i, sec[i].tolist(), sa[i].tolist(), sta[i].tolist(), sb[i].tolist(), stb[i].tolist())
(ea, ta), (eb, tb) = res
diff = np.flatnonzero(np.any(ea != eb, axis=1) | np.any(ta != tb, axis=1))
print(json.dumps({"rays": len(rays), "differ": int(diff.size)}))
for i in diff[:8]:
    print(i, rays[i].tolist(), ea[i].tolist(), ta[i].tolist(), eb[i].tolist(), tb[i].tolist())
