"""Independent restatement of the reference's scene loading for the hot path
(TEST INFRASTRUCTURE: shares no code with igx's C++ loader, host/scene_loader.cpp).

The oracle renders from the `igx_scene_desc` that igx's loader builds, so a
loader error (camera basis, entity transforms, plane-light axes, materials)
would show up identically in the GPU and the oracle images.  This module reads
the same JSON files the way the reference's runtime does and `check_desc`
compares its result with igx's descriptor field by field:

* externals and replace-by-name: Parser.cpp:395-459, Scene.cpp:5-23;
* transforms: Parser.cpp:116-232 (row-major 9/12/16 arrays; op lists
  translate / scale / rotate / qrotate / lookat / matrix, right-multiplied in
  order; lookAt :142-162), made affine (LoaderEntity.cpp:134);
* camera: PerspectiveCamera.cpp:8-23 and getOrientation (:67-75: eye = T*0,
  dir = T.col(2), up = T.col(1)), Camera.cpp:5-15 (vfov / hfov / fov);
* technique: PathTechnique.cpp / Technique.h defaults (max_depth 64,
  min_depth 2, clamp 0, nee on);
* entities: grouped by material in first-appearance order, an area-lit entity
  gets its own material (LoaderEntity.cpp:42-103); to_local / to_global /
  inverse-transpose normal matrix (:150-160);
* shapes: PLY (ascii / binary little endian) and OBJ read here, procedural
  rectangles from TriMeshProvider.cpp:27-41; shape `transform`
  (TriMeshProvider.cpp:540-541);
* area lights: plane representation when the mesh is a 4-vertex, 2-face
  parallelogram (TriMesh::getAsPlane, TriMesh.cpp:520-...), compared as the
  set of its four world corners, its normal (the mesh's face orientation) and
  its area (AreaLight.cpp:59-70); point / spot / env lights by their
  parameters (PointLight.cpp, SpotLight.cpp, EnvironmentLight.cpp).
"""
import json
import math
import os
import struct

import numpy as np

NAMED = ("shapes", "textures", "bsdfs", "lights", "media", "entities")
ANON = ("camera", "technique", "film")


# ------------------------------------------------------------------ parsing
def _put(lst, obj):
    for i, o in enumerate(lst):
        if o["name"] == obj["name"]:
            lst[i] = obj
            return
    lst.append(obj)


def load_json_scene(path):
    """-> dict with the merged scene (Parser.cpp:450-459 + Scene::addFrom)."""
    path = os.path.abspath(path)
    with open(path) as f:
        doc = json.load(f)
    base = os.path.dirname(path)
    scene = {k: [] for k in NAMED}
    for ext in doc.get("externals", []):
        sub = load_json_scene(os.path.join(base, ext["filename"]))
        for k in NAMED:
            for o in sub[k]:
                _put(scene[k], o)
        for k in ANON:  # taken from the external, even when it has none
            scene[k] = sub.get(k)
    for k in ANON:
        if k in doc:
            scene[k] = doc[k]
    for k in NAMED:
        for o in doc.get(k, []):
            o = dict(o)
            o.setdefault("__dir", base)
            _put(scene[k], o)
    return scene


def _vec(v, default=None):
    if v is None:
        return np.array(default, np.float64)
    if isinstance(v, (int, float)):
        return np.array([v, v, v], np.float64)
    if isinstance(v, str):
        # a PExpr colour expression (ShadingTree::computeColor) in its constant
        # forms: a number, color(v), color(r, g, b), color(r, g, b, a)
        import re
        m = re.fullmatch(r"\s*color\s*\(([^()]*)\)\s*", v)
        vals = [float(x) for x in (m.group(1).split(",") if m else [v])]
        if len(vals) not in (1, 3, 4):
            raise ValueError(f"not a constant colour: {v!r}")
        return np.array(vals[:3] if len(vals) > 1 else vals * 3, np.float64)
    return np.array(list(v) + [0] * (3 - len(v)), np.float64)


def _rot(axis, a):
    c, s = math.cos(a), math.sin(a)
    m = np.eye(4)
    i, j = [(1, 2), (0, 2), (0, 1)][axis]
    m[i, i], m[i, j], m[j, i], m[j, j] = c, -s, s, c
    if axis == 1:
        m[i, j], m[j, i] = s, -s
    return m


def _look_at(eye, center, up):
    f = center - eye
    f = f / np.linalg.norm(f) if np.linalg.norm(f) > 0 else np.array([0, 0, 1.0])
    u = up / np.linalg.norm(up)
    s = np.cross(f, u)
    s /= np.linalg.norm(s)
    u = np.cross(s, f)
    m = np.eye(4)
    m[:3, 0], m[:3, 1], m[:3, 2], m[:3, 3] = s, u, f, eye
    return m


def transform(v):
    """Parser.cpp getProperty / getTransform -> 4x4 float64."""
    t = np.eye(4)
    if v is None:
        return t
    if isinstance(v, dict):
        v = [v]
    if len(v) and isinstance(v[0], dict):
        for op in v:
            for k, a in op.items():
                if k == "translate":
                    m = np.eye(4)
                    m[:3, 3] = _vec(a)
                elif k == "scale":
                    m = np.diag(list(_vec(a)) + [1.0])
                elif k == "rotate":
                    a = np.radians(_vec(a))
                    m = _rot(0, a[0]) @ _rot(1, a[1]) @ _rot(2, a[2])
                elif k == "qrotate":
                    w, x, y, z = np.array(a, np.float64) / np.linalg.norm(a)
                    m = np.eye(4)
                    m[:3, :3] = [[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                                 [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                                 [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]]
                elif k == "lookat":
                    o = _vec(a.get("origin"), [0, 0, 0])
                    up = _vec(a.get("up"), [0, 0, 1])
                    tgt = o + _vec(a["direction"]) if "direction" in a else _vec(a.get("target"), [0, 1, 0])
                    m = _look_at(o, tgt, up)
                elif k == "matrix":
                    m = transform(a)
                else:
                    raise ValueError(k)
                t = t @ m
        return t
    n = len(v)
    if n == 9:
        t[:3, :3] = np.array(v, np.float64).reshape(3, 3)
    elif n in (12, 16):
        t[:n // 4, :] = np.array(v, np.float64).reshape(n // 4, 4)
    else:
        raise ValueError(f"transform of {n} entries")
    return t


# ------------------------------------------------------------------ meshes
_PLY_TYPES = {"float": "f", "float32": "f", "double": "d", "float64": "d", "uchar": "B", "uint8": "B", "char": "b",
              "int8": "b", "short": "h", "int16": "h", "ushort": "H", "uint16": "H", "int": "i", "int32": "i",
              "uint": "I", "uint32": "I"}


def read_ply(path):
    with open(path, "rb") as f:
        data = f.read()
    end = data.index(b"end_header") + len(b"end_header")
    end = data.index(b"\n", end) + 1
    header = data[:end].decode("ascii", "replace").splitlines()
    fmt = [l.split()[1] for l in header if l.startswith("format")][0]
    elems = []
    for l in header:
        p = l.split()
        if p[:1] == ["element"]:
            elems.append([p[1], int(p[2]), []])
        elif p[:1] == ["property"]:
            elems[-1][2].append(p[1:])
    verts, faces = None, []
    toks, pos = (data[end:].split(), 0) if fmt == "ascii" else (None, end)
    assert fmt in ("ascii", "binary_little_endian"), fmt

    def scalar(t):
        nonlocal pos
        if toks is not None:
            pos += 1
            return float(toks[pos - 1])
        f = "<" + _PLY_TYPES[t]
        pos += struct.calcsize(f)
        return struct.unpack_from(f, data, pos - struct.calcsize(f))[0]

    for name, cnt, props in elems:
        rows = []
        for _ in range(cnt):
            row = []
            for pr in props:
                if pr[0] == "list":
                    k = int(scalar(pr[1]))
                    row.append([scalar(pr[2]) for _ in range(k)])
                else:
                    row.append(scalar(pr[0]))
            rows.append(row)
        if name == "vertex":
            names = [p[-1] for p in props]
            verts = np.array([[r[names.index(c)] for c in "xyz"] for r in rows], np.float64)
        elif name == "face":
            faces = [[int(i) for i in r[0]] for r in rows]
    tris = [(f[0], f[k], f[k + 1]) for f in faces for k in range(1, len(f) - 1)]  # fan triangulation
    return verts, np.array(tris, np.int64)


def read_obj(path):
    verts, tris = [], []
    with open(path) as f:
        for line in f:
            p = line.split()
            if not p:
                continue
            if p[0] == "v":
                verts.append([float(x) for x in p[1:4]])
            elif p[0] == "f":
                idx = [int(t.split("/")[0]) for t in p[1:]]
                idx = [i - 1 if i > 0 else len(verts) + i for i in idx]
                tris += [(idx[0], idx[k], idx[k + 1]) for k in range(1, len(idx) - 1)]
    return np.array(verts, np.float64), np.array(tris, np.int64)


def shape_mesh(shape):
    """(vertices, triangles) in shape space, or None for non-mesh / unsupported shapes."""
    typ = shape.get("type")
    if typ in ("ply", "obj", "external"):
        fn = os.path.join(shape["__dir"], shape["filename"])
        v, t = read_ply(fn) if fn.lower().endswith(".ply") else read_obj(fn)
    elif typ == "rectangle" and "p0" not in shape:
        w, h = shape.get("width", 2.0), shape.get("height", 2.0)
        o = _vec(shape.get("origin"), [-w / 2, -h / 2, 0])
        X, Y = np.array([w, 0, 0.0]), np.array([0, h, 0.0])
        v = np.array([o, o + X, o + X + Y, o + Y])
        t = np.array([(0, 1, 2), (0, 2, 3)])
    else:
        return None
    if shape.get("flip_normals", False):
        t = t[:, [0, 2, 1]]
    st = transform(shape.get("transform"))
    v = v @ st[:3, :3].T + st[:3, 3]
    return v, t


def as_plane(v, t):
    """Plane test of TriMesh::getAsPlane: exactly 4 vertices and 2 faces with the
    same orientation and matching edge lengths -> (corners, unit normal)."""
    if len(t) != 2 or len(v) != 4:
        return None
    n = [np.cross(v[f[1]] - v[f[0]], v[f[2]] - v[f[0]]) for f in t]
    n = [x / np.linalg.norm(x) for x in n]
    if np.linalg.norm(n[0] - n[1]) > 1e-5:
        return None
    e = lambda f: [np.sum((v[f[i]] - v[f[(i + 1) % 3]]) ** 2) for i in range(3)]
    e0, e1 = e(t[0]), e(t[1])
    if not all(any(abs(a - b) <= 1e-5 for a in e0) for b in e1):
        return None
    return v, n[0]


# ------------------------------------------------------------------ scene
def interpret(path):
    """Everything check_desc compares, from the JSON alone."""
    sc = load_json_scene(path)
    film = (sc.get("film") or {}).get("size", [800, 600])
    tech = sc.get("technique") or {}
    cam = sc.get("camera") or {}
    out = {
        "film": (int(film[0]), int(film[1])),
        "technique": (int(tech.get("max_depth", 64)), int(tech.get("min_depth", 2)),
                      float(tech.get("clamp", 0.0)), bool(tech.get("nee", True))),
        "light_selector": tech.get("light_selector", ""),
    }
    if "vfov" in cam:
        fov, vert = cam["vfov"], True
    else:
        fov, vert = cam.get("hfov", cam.get("fov", 60.0)), False
    near, far = float(cam.get("near_clip", 0.0)), float(cam.get("far_clip", 3.4028234664e38))
    if far < near:
        near, far = far, near
    out["camera"] = {"fov": math.radians(fov), "vertical": vert, "near": near, "far": far}
    if "transform" in cam:
        T = transform(cam["transform"])
        out["camera"].update(eye=T[:3, 3], dir=T[:3, 2], up=T[:3, 1])

    area_entities = {l["entity"]: l for l in sc["lights"] if l.get("type") == "area"}
    bsdfs = {b["name"]: b for b in sc["bsdfs"]}
    shapes = {s["name"]: s for s in sc["shapes"]}
    groups = []  # (bsdf name, area entity or None, [entities])
    for e in sc["entities"]:
        if e["name"] in area_entities:
            groups.append((e["bsdf"], e["name"], [e]))
            continue
        for g in groups:
            if g[0] == e["bsdf"] and g[1] is None:
                g[2].append(e)
                break
        else:
            groups.append((e["bsdf"], None, [e]))
    ents, ent_index = [], {}
    for mid, (bname, _, members) in enumerate(groups):
        for e in members:
            T = transform(e.get("transform"))
            T[3] = [0, 0, 0, 1]
            ent_index[e["name"]] = len(ents)
            ents.append({"name": e["name"], "material": mid, "bsdf": bsdfs[bname], "to_global": T[:3],
                         "to_local": np.linalg.inv(T)[:3], "normal": np.linalg.inv(T[:3, :3]).T,
                         "shape": shapes[e["shape"]]})
    out["entities"] = ents

    lights = []
    for l in sc["lights"]:
        typ = l.get("type")
        if typ == "area":
            e = ents[ent_index[l["entity"]]]
            rec = {"type": "area", "entity": ent_index[l["entity"]], "radiance": _vec(l.get("radiance", 1.0)),
                   "power": "power" in l}
            m = shape_mesh(e["shape"])
            pl = as_plane(*m) if m is not None and l.get("optimize", True) else None
            if pl is not None:
                corners, n = pl
                T = e["to_global"]
                wc = corners @ T[:, :3].T + T[:, 3]
                wn = np.linalg.det(T[:, :3]) * (np.linalg.inv(T[:, :3]).T @ n)  # orientation of the mapped face
                rec.update(plane=True, corners=wc, normal=wn / np.linalg.norm(wn))
                # Light::position / computeFlux of a plane emitter (AreaLight.cpp:66-69, 99-113)
                area = np.linalg.norm(np.cross(wc[1] - wc[0], wc[2] - wc[0]))
                if np.abs(np.dot(wc[3] - wc[0], wc[3] - wc[0]) - np.dot(wc[1] - wc[0], wc[1] - wc[0])
                          - np.dot(wc[2] - wc[0], wc[2] - wc[0])) > 1e-3 * max(1.0, area):
                    area = np.linalg.norm(np.cross(wc[1] - wc[0], wc[3] - wc[0]))  # corner order of the diagonal
                rec.update(select_position=wc.mean(axis=0), select_flux=float(np.mean(rec["radiance"])) * area * math.pi)
            else:
                rec["plane"] = False
            lights.append(rec)
        elif typ in ("env", "constant", "uniform"):
            lights.append({"type": "env", "radiance": _vec(l.get("radiance", 1.0)) * _vec(l.get("scale", 1.0))})
        elif typ == "point":
            # PointLight.cpp:16-30, 61-69: `power` P gives the intensity P / (4 pi)
            if "power" in l:
                P = _vec(l["power"])
                I = P / (4 * math.pi)
            else:
                I = _vec(l.get("intensity", 1.0))
                P = I * 4 * math.pi
            lights.append({"type": "point", "position": _vec(l.get("position"), [0, 0, 0]), "intensity": I,
                           "select_flux": float(np.mean(P))})
        elif typ == "spot":
            d = _vec(l.get("direction"), [0, 0, 1])
            c_, f_ = math.radians(l.get("cutoff", 30)), math.radians(l.get("falloff", 20))
            I = _vec(l.get("intensity", 1.0))
            lights.append({"type": "spot", "position": _vec(l.get("position"), [0, 0, 0]),
                           "direction": d / np.linalg.norm(d), "intensity": I, "cutoff": c_, "falloff": f_,
                           # SpotLight.cpp:17-38
                           "select_flux": float(np.mean(I)) * 2 * math.pi * (1 - 0.5 * (math.cos(c_) + math.cos(f_)))})
        else:
            lights.append({"type": typ})
    out["lights"] = lights  # file order (the device puts infinite lights first itself)
    return out


# ------------------------------------------------------------------ comparison
BSDF_TYPES = {"diffuse": 0, "dielectric": 1, "glass": 1, "conductor": 2, "roughconductor": 2, "mirror": 2,
              "plastic": 3, "roughplastic": 3, "principled": 4}  # IGX_BSDF_* (include/igx_scene.h)


def _close(a, b, what, rtol=1e-5, atol=1e-4):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    if a.shape != b.shape or not np.allclose(a, b, rtol=rtol, atol=atol):
        raise AssertionError(f"{what}: igx {a.tolist()} vs reference reading {b.tolist()}")


def _check_light(i, L, rl, desc):
    if rl["type"] == "area":
        if L.entity != rl["entity"]:
            raise AssertionError(f"light {i}: entity {L.entity} vs {rl['entity']}")
        if not rl["power"]:
            _close(L.radiance[:], rl["radiance"], f"light {i} radiance")
        if rl["plane"]:
            if L.type != 1:
                raise AssertionError(f"light {i}: type {L.type}, expected a plane emitter")
            o, X, Y = np.array(L.origin[:]), np.array(L.x_axis[:]), np.array(L.y_axis[:])
            got = np.array([o, o + X, o + Y, o + X + Y])
            for p in rl["corners"]:
                if np.min(np.linalg.norm(got - p, axis=1)) > 1e-3 * max(1.0, np.abs(p).max()):
                    raise AssertionError(f"light {i}: plane corner {p.tolist()} not in {got.tolist()}")
            _close(L.normal[:], rl["normal"], f"light {i} plane normal")
            _close([L.area], [np.linalg.norm(np.cross(X, Y))], f"light {i} area")
            _close(L.select_position[:], rl["select_position"], f"light {i} selector position")
            _close(L.select_direction[:], rl["normal"], f"light {i} selector direction")
            if not rl["power"]:
                _close([L.select_flux], [rl["select_flux"]], f"light {i} selector flux", rtol=1e-4)
        elif L.type == 1:
            raise AssertionError(f"light {i}: plane emitter for a non-plane mesh")
    elif rl["type"] == "env":
        if L.type != 2:
            raise AssertionError(f"light {i}: type {L.type}, expected env")
        _close(L.radiance[:], rl["radiance"], f"light {i} radiance")
    elif rl["type"] == "point":
        if L.type != 3:
            raise AssertionError(f"light {i}: type {L.type}, expected point")
        _close(L.origin[:], rl["position"], f"light {i} position")
        _close(L.radiance[:], rl["intensity"], f"light {i} intensity")
        _close(L.select_position[:], rl["position"], f"light {i} selector position")
        _close([L.select_flux], [rl["select_flux"]], f"light {i} selector flux", rtol=1e-4)
        if L.select_has_direction:
            raise AssertionError(f"light {i}: a point light has no direction")
    elif rl["type"] == "spot":
        if L.type != 4:
            raise AssertionError(f"light {i}: type {L.type}, expected spot")
        _close(L.origin[:], rl["position"], f"light {i} position")
        _close(L.normal[:], rl["direction"], f"light {i} direction")
        _close(L.radiance[:], rl["intensity"], f"light {i} intensity")
        _close([L.cutoff, L.falloff], [rl["cutoff"], rl["falloff"]], f"light {i} cone")
        _close(L.select_direction[:], rl["direction"], f"light {i} selector direction")
        _close([L.select_flux], [rl["select_flux"]], f"light {i} selector flux", rtol=1e-4)


def check_desc(path, desc):
    """Raise AssertionError on the first field where igx's descriptor differs
    from this independent reading of the scene file."""
    ref = interpret(path)
    if (desc.film_width, desc.film_height) != ref["film"]:
        raise AssertionError(f"film {desc.film_width}x{desc.film_height} vs {ref['film']}")
    t = desc.technique
    if (t.max_depth, t.min_depth, t.nee != 0) != (ref["technique"][0], ref["technique"][1], ref["technique"][3]):
        raise AssertionError(f"technique {(t.max_depth, t.min_depth, t.nee)} vs {ref['technique']}")
    _close(t.clamp, ref["technique"][2], "technique.clamp")
    # LoaderLight::generateLightSelector (LoaderLight.cpp:423-453): "hierarchy", "simple", else uniform
    sel = ref["light_selector"]
    if t.light_selector != {"hierarchy": 2, "simple": 1}.get(sel, 0):
        raise AssertionError(f"technique.light_selector {t.light_selector} vs '{sel}'")
    c, rc = desc.camera, ref["camera"]
    _close(c.fov, rc["fov"], "camera.fov", rtol=1e-6)
    if bool(c.vertical_fov) != rc["vertical"]:
        raise AssertionError("camera fov axis")
    _close([c.near_clip], [rc["near"]], "camera.near_clip")
    if rc["far"] < 1e37:
        _close([c.far_clip], [rc["far"]], "camera.far_clip")
    if "eye" in rc:
        _close(c.eye[:], rc["eye"], "camera.eye")
        _close(c.dir[:], rc["dir"], "camera.dir")
        _close(c.up[:], rc["up"], "camera.up")
    if desc.num_entities != len(ref["entities"]):
        raise AssertionError(f"{desc.num_entities} entities vs {len(ref['entities'])}")
    for i, re_ in enumerate(ref["entities"]):
        e = desc.entities[i]
        if e.material != re_["material"]:
            raise AssertionError(f"entity {re_['name']}: material {e.material} vs {re_['material']}")
        _close(np.array(e.to_global[:]).reshape(3, 4), re_["to_global"], f"entity {re_['name']} to_global")
        _close(np.array(e.to_local[:]).reshape(3, 4), re_["to_local"], f"entity {re_['name']} to_local", atol=1e-3)
        _close(np.array(e.normal[:]).reshape(3, 3), re_["normal"], f"entity {re_['name']} normal matrix", atol=1e-3)
        b = re_["bsdf"]
        m = desc.materials[e.material]
        bt = BSDF_TYPES.get(b.get("type"))
        if bt is not None and m.bsdf_type != bt:
            raise AssertionError(f"entity {re_['name']}: bsdf type {m.bsdf_type} vs {b.get('type')}")
        refl = b.get("reflectance", 0.8)
        if b.get("type") == "diffuse" and isinstance(refl, str) and "checkerboard" in refl:
            # select(checkerboard(uvw * S) == 1, A, B): texture/checkerboard.art, Transpiler.cpp
            import re
            mm = re.fullmatch(r"\s*select\(\s*checkerboard\(\s*uvw\s*\*\s*([-+0-9.eE]+)\s*\)\s*==\s*1\s*,"
                              r"\s*(color\([^()]*\))\s*,\s*(color\([^()]*\))\s*\)\s*", refl)
            if not mm:
                raise AssertionError(f"bsdf {b['name']}: unexpected texture expression {refl!r}")
            if m.texture != 1:
                raise AssertionError(f"bsdf {b['name']}: texture {m.texture}, expected the checker")
            _close([m.tex_scale], [float(mm.group(1))], f"bsdf {b['name']} checker scale")
            _close(m.tex_kd1[:], _vec(mm.group(2)), f"bsdf {b['name']} checker colour 1")
            _close(m.kd[:], _vec(mm.group(3)), f"bsdf {b['name']} checker colour 0")
        elif b.get("type") == "diffuse":
            if m.texture != 0:
                raise AssertionError(f"bsdf {b['name']}: texture {m.texture} on a plain colour")
            _close(m.kd[:], _vec(refl), f"bsdf {b['name']} reflectance")
        if b.get("type") in ("dielectric", "glass"):
            if "int_ior" in b:
                _close([m.int_ior], [b["int_ior"]], f"bsdf {b['name']} int_ior")
            if "ext_ior" in b:
                _close([m.ext_ior], [b["ext_ior"]], f"bsdf {b['name']} ext_ior")
            if bool(m.thin) != bool(b.get("thin", False)):
                raise AssertionError(f"bsdf {b['name']} thin")
    if desc.num_lights != len(ref["lights"]):
        raise AssertionError(f"{desc.num_lights} lights vs {len(ref['lights'])}")
    for i, rl in enumerate(ref["lights"]):
        _check_light(i, desc.lights[i], rl, desc)
    for i in range(desc.num_entities):
        m = desc.materials[desc.entities[i].material]
        if m.light >= 0 and desc.lights[m.light].entity != i:
            raise AssertionError(f"entity {i}: emitting material points at light {m.light} of another entity")
    return ref
