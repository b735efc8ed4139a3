"""Dev probe: traversal cost of a scene's two-level BVH (TLAS over entities,
BLAS per mesh) against one flat BVH over the same triangles in world space.
Writes the flattened scene as one OBJ entity, traces the same rays through
both with igx_trace_hits (kernel time via the timing option) and compares the
hit distances.
usage: flat_probe.py [scene.json] [n_random_rays]"""
import json, os, sys, tempfile, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ignis-masterthesis_amd"))
import ignis_amd

path = os.path.join(ROOT, sys.argv[1] if len(sys.argv) > 1 else "scenes/diamond_scene.json")
nrand = int(sys.argv[2]) if len(sys.argv) > 2 else 4_000_000
scene = ignis_amd.Scene.from_file(path)
d = scene.desc
verts, faces = [], []
base = 0
for e in range(d.num_entities):
    en = d.entities[e]
    sh = d.shapes[en.shape]
    if sh.type != 0:
        continue
    m = d.meshes[sh.mesh]
    v = np.ctypeslib.as_array(m.vertices, (m.num_vertices * 3,)).reshape(-1, 3).astype(np.float64)
    f = np.ctypeslib.as_array(m.indices, (m.num_faces * 3,)).reshape(-1, 3)
    T = np.array(list(en.to_global), np.float64).reshape(3, 4)
    w = v @ T[:, :3].T + T[:, 3]
    verts.append(w.astype(np.float32))
    faces.append(f + base)
    base += len(v)
verts = np.concatenate(verts)
faces = np.concatenate(faces)
tmp = tempfile.mkdtemp()
with open(os.path.join(tmp, "flat.obj"), "w") as fo:
    for p in verts:
        fo.write(f"v {p[0]:.9g} {p[1]:.9g} {p[2]:.9g}\n")
    for f in faces:
        fo.write(f"f {f[0] + 1} {f[1] + 1} {f[2] + 1}\n")
c = d.camera
flat = {"technique": {"type": "path", "max_depth": 2},
        "camera": {"type": "perspective", "fov": float(np.degrees(c.fov)), "near_clip": c.near_clip, "far_clip": c.far_clip,
                   "transform": [1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0]},
        "film": {"size": [d.film_width, d.film_height]},
        "bsdfs": [{"name": "w", "type": "diffuse"}],
        "shapes": [{"name": "flat", "type": "obj", "filename": "flat.obj"}],
        "entities": [{"name": "flat", "shape": "flat", "bsdf": "w"}]}
fscene = ignis_amd.Scene.from_string(json.dumps(flat), tmp)

# rays: camera rays of the film, random rays from inside the scene box, and
# rays from inside the smallest entity boxes (the diamonds' interior bounces)
rng = np.random.default_rng(3)
lo, hi = np.array(list(d.scene_bbox_min)), np.array(list(d.scene_bbox_max))
W, H = d.film_width, d.film_height
eye, dr, up = np.array(c.eye[:]), np.array(c.dir[:]), np.array(c.up[:])
right = np.cross(dr, up); right /= np.linalg.norm(right)
sx = np.tan(c.fov / 2); sy = sx / (W / H)
ys, xs = np.mgrid[0:H, 0:W]
v = sx * (2 * (xs + 0.5) / W - 1)[..., None] * right + sy * (1 - 2 * (ys + 0.5) / H)[..., None] * up + dr
v = (v / np.linalg.norm(v, axis=-1, keepdims=True)).reshape(-1, 3)
cam = np.zeros((len(v), 8), np.float32)
cam[:, 0:3], cam[:, 3:6], cam[:, 6], cam[:, 7] = eye, v, c.near_clip, c.far_clip
boxes = [(np.array(list(d.entities[e].bbox_min)), np.array(list(d.entities[e].bbox_max))) for e in range(d.num_entities)]
vol = [np.prod(np.maximum(b - a, 1e-6)) for a, b in boxes]
small = [boxes[i] for i in np.argsort(vol)[:3]]
def rand_rays(n, a, b):
    r = np.zeros((n, 8), np.float32)
    r[:, 0:3] = a + (b - a) * rng.random((n, 3))
    dd = rng.normal(size=(n, 3)); dd /= np.linalg.norm(dd, axis=1, keepdims=True)
    r[:, 3:6], r[:, 6], r[:, 7] = dd, 1e-3, 1e30
    return r
sets = {"camera": cam, "box": rand_rays(nrand, lo, hi),
        "inside_small": np.concatenate([rand_rays(nrand // 3, a, b) for a, b in small])}
dev = ignis_amd.Device(0)
res = {}
for name, sc in (("two_level", scene), ("flat", fscene)):
    dev.upload(sc)
    s0 = dev.stats()
    out = {"depth": s0["bvh_depth"], "width": s0["bvh_width"]}
    for rn, rays in sets.items():
        dev.trace_hits(rays[:1024])
        dev.reset_stats(); dev.set_option("timing", 1)
        for _ in range(3):
            ep, tuv = dev.trace_hits(rays)
        st = dev.stats(); dev.set_option("timing", 0)
        out[rn + "_ms"] = round(st["ms_trace"] / 3, 3)
        out[rn + "_t"] = tuv[:, 0].copy()
        out[rn + "_hit"] = ep[:, 0] >= 0
    res[name] = out
for rn in sets:
    a, b = res["two_level"], res["flat"]
    same = np.mean((a[rn + "_hit"] == b[rn + "_hit"]) & (np.abs(a[rn + "_t"] - b[rn + "_t"]) <= 1e-5 * np.abs(a[rn + "_t"]) + 1e-7))
    print(json.dumps({"rays": rn, "n": len(sets[rn]), "two_level_ms": a[rn + "_ms"], "flat_ms": b[rn + "_ms"],
                      "speedup": round(a[rn + "_ms"] / max(b[rn + "_ms"], 1e-9), 3), "t_agree": round(float(same), 5)}))
print(json.dumps({"two_level": {k: v for k, v in res["two_level"].items() if k in ("depth", "width")},
                  "flat": {k: v for k, v in res["flat"].items() if k in ("depth", "width")}, "flat_tris": int(len(faces))}))
