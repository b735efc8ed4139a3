"""Freeze the procedural geometry igx generates into tests/golden/procedural_shapes.npz.

The reference's procedural shapes (src/runtime/mesh/TriMesh.cpp: MakePlane,
MakeRectangle, MakeBox, MakeIcoSphere, MakeUVSphere, MakeCylinder, MakeCone,
MakeDisk) and its plane / sphere detection (getAsPlane / getAsSphere) decide
the exact triangles and emitters the hot path intersects, so their output is
pinned as data: vertices, normals, texture coordinates and faces of every
procedural shape the scenes use, plus the plane and sphere detection results
for the scene meshes.  tests/test_loader_abi.py checks the library against
this file bit for bit.

Generated once from the library (python tests/golden/make_shape_fixture.py);
regenerate only for an intended geometry change.
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "ignis-masterthesis_amd"), ROOT]

SHAPES = {
    "rect": {"type": "rectangle", "width": 3, "height": 2},
    "rect_flip": {"type": "rectangle", "width": 2, "height": 2, "flip_normals": True},
    "rect_p": {"type": "rectangle", "p0": [0, 0, 0], "p1": [2, 0, 0], "p2": [2, 1, 0.5], "p3": [0, 1, 0.5]},
    "tri": {"type": "triangle", "p0": [0, 0, 0], "p1": [1, 0, 0], "p2": [0, 2, 1]},
    "cube": {"type": "cube", "width": 8, "height": 8, "depth": 8, "flip_normals": True},
    "box": {"type": "box", "width": 1, "height": 2, "depth": 3, "origin": [0.5, 0, -1]},
    "ico0": {"type": "icosphere", "subdivisions": 0},
    "ico2": {"type": "icosphere", "center": [1, 2, 3], "radius": 0.5, "subdivisions": 2},
    "ico5": {"type": "icosphere", "subdivisions": 5},
    "uv": {"type": "uvsphere", "center": [0, 0, 1], "radius": 2, "stacks": 8, "slices": 6},
    "uv_default": {"type": "uvsphere"},
    "cyl": {"type": "cylinder"},
    "cyl_open": {"type": "cylinder", "p0": [0, 0, -1], "p1": [0, 1, 1], "bottom_radius": 0.5, "top_radius": 0.25,
                 "sections": 7, "filled": False},
    "cone": {"type": "cone", "radius": 0.75, "p1": [0, 0, 2], "sections": 9},
    "disk": {"type": "disk", "origin": [0, 1, 0], "normal": [0, 1, 0], "radius": 2, "sections": 12},
    "disk_tilted": {"type": "disk", "normal": [0.3, -0.4, 0.866], "sections": 5},
}
MESH_FILES = ["scenes/meshes/Bottom.ply", "scenes/meshes/Top.ply", "scenes/meshes/Back.ply",
              "scenes/meshes/Diamond.ply", "scenes/evaluation/meshes/cbox_luminaire.obj",
              "scenes/evaluation/meshes/cbox_ceiling.obj", "scenes/evaluation/meshes/cbox_floor.obj",
              "scenes/evaluation/meshes/cbox_largebox.obj", "scenes/evaluation/meshes/IcosphereHQ.ply",
              "scenes/evaluation/meshes/Plane.ply", "scenes/meshes/Room.obj"]


def mesh_arrays(desc, i):
    m = desc.meshes[i]
    nv, nf = m.num_vertices, m.num_faces
    v = np.ctypeslib.as_array(m.vertices, shape=(nv * 3,)).copy()
    n = np.ctypeslib.as_array(m.normals, shape=(nv * 3,)).copy()
    t = np.ctypeslib.as_array(m.texcoords, shape=(nv * 2,)).copy()
    f = np.ctypeslib.as_array(m.indices, shape=(nf * 3,)).copy()
    return v, n, t, f


def scene_for(shapes):
    return {
        "technique": {"type": "path", "max_depth": 2},
        "camera": {"type": "perspective", "fov": 60, "transform": [1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, -10]},
        "film": {"size": [8, 8]},
        "bsdfs": [{"type": "diffuse", "name": "d"}],
        "shapes": shapes,
        "entities": [{"name": "e" + s["name"], "shape": s["name"], "bsdf": "d"} for s in shapes],
        "lights": [{"type": "area", "name": "l" + s["name"], "entity": "e" + s["name"]} for s in shapes],
    }


def generate():
    import ignis_amd

    out = {}
    shapes = [dict(v, name=k) for k, v in SHAPES.items()]
    files = [{"type": "external", "name": os.path.basename(f).replace(".", "_"), "filename": os.path.join(ROOT, f)}
             for f in MESH_FILES if os.path.exists(os.path.join(ROOT, f))]
    sc = ignis_amd.Scene.from_string(json.dumps(scene_for(shapes + files)), ROOT)
    d = sc.desc
    names = [s["name"] for s in shapes + files]
    for i, name in enumerate(names):
        sh = d.shapes[d.entities[i].shape]
        v, n, t, f = mesh_arrays(d, sh.mesh)
        if name in SHAPES:
            out[f"{name}/vertices"], out[f"{name}/normals"], out[f"{name}/texcoords"], out[f"{name}/faces"] = v, n, t, f
        out[f"{name}/is_plane"] = np.array([sh.is_plane], np.int32)
        out[f"{name}/plane"] = np.array(list(sh.plane_origin) + list(sh.plane_x) + list(sh.plane_y) + list(sh.plane_tex),
                                        np.float32)
        L = d.lights[i]
        out[f"{name}/light"] = np.array([L.type] + list(L.origin) + [L.radius, L.area], np.float32)
    return out


if __name__ == "__main__":
    data = generate()
    path = os.path.join(ROOT, "tests", "golden", "procedural_shapes.npz")
    np.savez_compressed(path, **data)
    print("wrote", path, len(data), "arrays", os.path.getsize(path), "bytes")
