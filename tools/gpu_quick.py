"""Quick GPU sanity run: hit parity + image parity on diamond vs the oracle (dev tool)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ignis-masterthesis_amd"))
sys.path.insert(0, ROOT)
import numpy as np
import ignis_amd
from oracle import oracle_py as O

scene = ignis_amd.Scene.from_file(os.path.join(ROOT, "scenes/diamond_scene.json"))
dev = ignis_amd.Device(0)
t = time.time(); dev.upload(scene); print("upload", time.time() - t, flush=True)
orc = O.OracleScene(scene)
# camera-like rays
rng = np.random.default_rng(1)
n = 20000
org = np.tile(np.array([0, 0, 3.85], np.float32), (n, 1))
d = rng.normal(size=(n, 3)).astype(np.float32); d[:, 2] = -np.abs(d[:, 2]) - 2.0
d /= np.linalg.norm(d, axis=1, keepdims=True)
rays = np.concatenate([org, d, np.full((n, 1), 0.1, np.float32), np.full((n, 1), 100, np.float32)], 1)
ep_g, tuv_g = dev.trace_hits(rays, 1)
ep_o, tuv_o = orc.trace_hits(rays, 1)
same = np.all(ep_g == ep_o, axis=1)
print("hit ids equal", same.mean(), "miss frac", (ep_o[:, 0] < 0).mean(), flush=True)
hit = same & (ep_o[:, 0] >= 0)
print("t rel err max", np.max(np.abs(tuv_g[hit, 0] - tuv_o[hit, 0]) / tuv_o[hit, 0]), flush=True)

W = H = 200
p = ignis_amd.RenderParams(); p.width, p.height, p.spi = W, H, 8
dev.set_option("timing", 1)
t = time.time(); dev.render(p); print("gpu render", time.time() - t, flush=True)
fb, it = dev.framebuffer(W * H * 3)
print("stats", dev.stats(), flush=True)
ofb, ost = orc.render(W, H, 8)
print("oracle stats", ost)
print("means gpu", fb.mean(), "oracle", ofb.mean(), flush=True)
diff = np.abs(fb - ofb)
print("exact-equal pixels", np.mean(diff == 0), "rel<1e-3", np.mean(diff <= 1e-3 * np.maximum(np.abs(ofb), 1e-3)), flush=True)
# full size timing
W, H = 1000, 1000
p.width, p.height = W, H
dev.reset_stats()
for i in range(3):
    p.iteration = i
    t = time.time(); dev.render(p); dt = time.time() - t
    print("1000^2 spi8 iter", i, "s", dt, flush=True)
s = dev.stats()
rays = s["camera_rays"] + s["bounce_rays"] + s["shadow_rays"]
print("Mrays/s (wall)", rays / (s["ms_render"] * 1e3), s, flush=True)
