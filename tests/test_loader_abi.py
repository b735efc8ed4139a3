"""Scene ingestion and the C-ABI surface (CPU only: no GPU calls)."""
import ctypes as C
import sys
import os
import re

import numpy as np
import pytest

import ignis_amd
from ignis_amd import _native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    names = set()
    for hdr in ("igx.h", "igx_scene.h"):
        text = open(os.path.join(ROOT, "include", hdr)).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        for m in re.finditer(r"\b(igx_[a-z_0-9]+)\s*\(", text):
            names.add(m.group(1))
    return sorted(names)


def test_library_exports_every_declared_symbol():
    lib = C.CDLL(_native.LIB_PATH)
    decl = declared_functions()
    assert len(decl) >= 15
    missing = [n for n in decl if not hasattr(lib, n)]
    assert not missing, missing
    assert sorted(_native.EXPORTED_SYMBOLS) == decl


def test_version_without_gpu():
    assert "gfx950" in ignis_amd.version()


def test_diamond_scene_tables(diamond_path):
    sc = ignis_amd.Scene.from_file(diamond_path)
    d = sc.desc
    assert (d.film_width, d.film_height) == (1000, 1000)
    assert d.num_entities == 9 and d.num_shapes == 7 and d.num_lights == 1
    # materials grouped per LoaderEntity.cpp:42-103: AreaLight gets its own
    assert d.num_materials == 4
    faces = [d.meshes[i].num_faces for i in range(d.num_meshes)]
    assert sum(faces) == 282  # 270 diamond + 5 walls x 2 + light 2
    inst = sum(d.meshes[d.shapes[d.entities[e].shape].mesh].num_faces for e in range(d.num_entities))
    assert inst == 822
    L = d.lights[0]
    assert L.type == 1  # plane emitter
    assert L.area == pytest.approx(0.04, rel=1e-3)
    n = np.array(L.normal[:])
    assert np.linalg.norm(n) == pytest.approx(1, abs=1e-6)
    # the area-light material references the light
    assert sum(1 for i in range(d.num_materials) if d.materials[i].light == 0) == 1
    assert d.technique.max_depth == 64 and d.technique.min_depth == 2
    cam = d.camera
    np.testing.assert_allclose(cam.eye[:], [0, 0, 3.85], atol=1e-6)
    np.testing.assert_allclose(cam.dir[:], [0, 0, -1])
    assert cam.fov == pytest.approx(np.deg2rad(40))


def test_primitives_scene_tables(primitives_path):
    sc = ignis_amd.Scene.from_file(primitives_path)
    d = sc.desc
    assert d.num_entities == 11 and d.num_lights == 1
    types = [d.shapes[i].type for i in range(d.num_shapes)]
    assert types.count(1) == 1  # "sphere" -> analytic SphereProvider (LoaderShape.cpp:24-40)
    assert d.lights[0].type == 2  # constant env
    assert d.technique.max_depth == 2
    # entity transform [{"translate":[-4,0,0]}, {"scale":0.5}] = T * S
    e = d.entities[4]
    m = np.array(e.to_global[:]).reshape(3, 4)
    np.testing.assert_allclose(m[:, :3], np.eye(3) * 0.5, atol=1e-7)
    np.testing.assert_allclose(m[:, 3], [-4, 0, 0], atol=1e-7)


def test_loader_errors_are_reported():
    with pytest.raises(ignis_amd.IgxError, match="unsupported shape type"):
        ignis_amd.Scene.from_string({"shapes": [{"type": "teapot", "name": "x"}]})
    with pytest.raises(ignis_amd.IgxError, match="unknown bsdf"):
        ignis_amd.Scene.from_string({"shapes": [{"type": "cube", "name": "c"}],
                                     "entities": [{"name": "e", "shape": "c", "bsdf": "nope"}]})
    with pytest.raises(ignis_amd.IgxError, match="JSON parse error"):
        ignis_amd.Scene.from_string("{ not json")
    with pytest.raises(ignis_amd.IgxError, match="cannot open"):
        ignis_amd.Scene.from_file("/nonexistent/scene.json")


def test_rectangle_flip_and_plane_detection():
    sc = ignis_amd.Scene.from_string({"shapes": [{"type": "rectangle", "name": "r", "flip_normals": True}]})
    d = sc.desc
    m = d.meshes[0]
    nrm = np.ctypeslib.as_array(m.normals, shape=(m.num_vertices * 3,)).reshape(-1, 3)
    np.testing.assert_allclose(nrm, np.tile([0, 0, -1], (4, 1)))
    s = d.shapes[0]
    assert s.is_plane == 1
    x = np.array(s.plane_x[:]); y = np.array(s.plane_y[:])
    assert np.cross(x, y) @ np.array([0, 0, -1]) > 0  # plane normal follows the (flipped) faces


def test_procedural_shapes_load():
    shapes = [{"type": t, "name": t} for t in ["cube", "icosphere", "uvsphere", "cylinder", "cone", "disk", "triangle"]]
    sc = ignis_amd.Scene.from_string({"shapes": shapes})
    d = sc.desc
    faces = {shapes[i]["type"]: d.meshes[d.shapes[i].mesh].num_faces for i in range(len(shapes))}
    assert faces["cube"] == 12
    assert faces["icosphere"] == 20 * 4 ** 4
    assert faces["triangle"] == 1
    assert faces["disk"] == 32
    for i in range(d.num_meshes):
        m = d.meshes[i]
        n = np.ctypeslib.as_array(m.normals, shape=(m.num_vertices * 3,)).reshape(-1, 3)
        np.testing.assert_allclose(np.linalg.norm(n, axis=1), 1, atol=1e-5)


def test_synthetic_bench_scenes(root):
    """SURVEY.md §8d stand-ins: soup size/extent and determinism, S-deep instancing."""
    soup = ignis_amd.Scene.from_file(os.path.join(root, "scenes", "s_soup_1m.json"))
    d = soup.desc
    assert d.num_meshes == 1 and d.meshes[0].num_faces == 1000000
    assert all(-1.011 < d.scene_bbox_min[i] < -0.99 and 0.99 < d.scene_bbox_max[i] < 1.011 for i in range(3))
    v = np.ctypeslib.as_array(d.meshes[0].vertices, shape=(9,)).copy()
    again = ignis_amd.Scene.from_file(os.path.join(root, "scenes", "s_soup_1m.json"))
    np.testing.assert_array_equal(v, np.ctypeslib.as_array(again.desc.meshes[0].vertices, shape=(9,)))
    # triangle edge length ~ e = 0.01 for 1M triangles
    t = v.reshape(3, 3)
    assert np.abs(t - t.mean(axis=0)).max() <= 0.02 + 1e-6
    deep = ignis_amd.Scene.from_file(os.path.join(root, "scenes", "s_deep.json"))
    dd = deep.desc
    assert dd.num_entities == 4097 and dd.num_meshes == 4
    faces = sorted(dd.meshes[i].num_faces for i in range(dd.num_meshes))
    assert faces == [2, 270, 20480, 131072]
    assert dd.num_lights == 2


def test_soup_and_grid_shapes_from_string():
    doc = {"shapes": [{"type": "soup", "name": "s", "count": 1000, "seed": 1},
                      {"type": "displaced_grid", "name": "g", "quads": 16, "size": 2.0, "amplitude": 0.5, "seed": 3}],
           "bsdfs": [{"type": "diffuse", "name": "d"}],
           "entities": [{"name": "a", "shape": "s", "bsdf": "d"}, {"name": "b", "shape": "g", "bsdf": "d"}]}
    sc = ignis_amd.Scene.from_string(doc)
    d = sc.desc
    counts = sorted(d.meshes[i].num_faces for i in range(d.num_meshes))
    assert counts == [512, 1000]
    with pytest.raises(ignis_amd.IgxError):
        ignis_amd.Scene.from_string({"shapes": [{"type": "soup", "name": "s", "count": 0}]})


def test_write_exr_roundtrip(tmp_path):
    """Image::save stand-in (Image.h:92-101): float RGB(A) EXR, read back by an independent parser."""
    from exr_read import read_exr
    rng = np.random.default_rng(5)
    img = rng.random((7, 11, 3), dtype=np.float32) * 10
    p = tmp_path / "out.exr"
    ignis_amd.write_exr(p, img, scale=0.5)
    ch, attrs = read_exr(p)
    assert sorted(ch) == ["B", "G", "R"]
    np.testing.assert_array_equal(ch["R"], img[..., 0] * 0.5)
    np.testing.assert_array_equal(ch["G"], img[..., 1] * 0.5)
    np.testing.assert_array_equal(ch["B"], img[..., 2] * 0.5)
    ignis_amd.write_exr(p, img, alpha=True)
    ch, _ = read_exr(p)
    assert sorted(ch) == ["A", "B", "G", "R"] and np.all(ch["A"] == 1)
    with pytest.raises(ignis_amd.IgxError):
        ignis_amd.write_exr(tmp_path / "missing_dir" / "x.exr", img)


def _emitter_doc(shape, light_extra=None, transform=None):
    ent = {"name": "E", "shape": "S", "bsdf": "d"}
    if transform:
        ent["transform"] = transform
    light = {"type": "area", "name": "L", "entity": "E", "radiance": [1, 2, 3]}
    light.update(light_extra or {})
    return {"bsdfs": [{"type": "diffuse", "name": "d"}], "shapes": [dict(shape, name="S")],
            "entities": [ent], "lights": [light]}


def _ellipsoid_area(l1, l2, l3, P):
    return 4 * np.pi * (((l1 * l2) ** P + (l1 * l3) ** P + (l2 * l3) ** P) / 3) ** (1 / P)


def test_area_light_representations():
    """AreaLight::AreaLight (AreaLight.cpp:38-99): plane -> plane sampler, analytic
    or mesh-detected sphere -> sphere sampler, any other triangle shape (or
    optimize=false) -> triangle-shape sampler."""
    keep = []

    def light_of(doc):
        sc = ignis_amd.Scene.from_string(doc)
        keep.append(sc)  # the desc is owned by the scene handle
        assert sc.desc.num_lights == 1
        return sc.desc.lights[0], sc.desc
    L, _ = light_of(_emitter_doc({"type": "rectangle"}))
    assert L.type == _native.LIGHT_PLANE
    L, _ = light_of(_emitter_doc({"type": "rectangle"}, {"optimize": False}))
    assert L.type == _native.LIGHT_MESH and L.entity == 0
    L, _ = light_of(_emitter_doc({"type": "cylinder"}))
    assert L.type == _native.LIGHT_MESH
    # analytic sphere, non-uniformly scaled: the emitter keeps the object-space sphere
    # and the P = 1.6 ellipsoid area of compute_ellipsoid_area (shapes/sphere.art:21-27)
    L, _ = light_of(_emitter_doc({"type": "sphere", "center": [1, 2, 3], "radius": 0.5},
                                 transform=[{"scale": [1, 2, 3]}]))
    assert L.type == _native.LIGHT_SPHERE
    np.testing.assert_allclose(L.origin[:], [1, 2, 3])
    assert L.radius == pytest.approx(0.5)
    assert L.area == pytest.approx(_ellipsoid_area(0.5, 1.0, 1.5, 1.6), rel=1e-5)
    # icosphere mesh: TriMesh::getAsSphere (TriMesh.cpp:636-698) detects the sphere
    L, _ = light_of(_emitter_doc({"type": "icosphere", "center": [0, 0, 1], "radius": 2, "subdivisions": 3}))
    assert L.type == _native.LIGHT_SPHERE
    np.testing.assert_allclose(L.origin[:], [0, 0, 1], atol=1e-5)
    assert L.radius == pytest.approx(2, rel=1e-5)
    assert L.area == pytest.approx(4 * np.pi * 4, rel=1e-5)
    # ... unless optimize = false: the mesh itself is sampled
    L, _ = light_of(_emitter_doc({"type": "icosphere", "subdivisions": 3}, {"optimize": False}))
    assert L.type == _native.LIGHT_MESH


def test_area_light_power():
    """'power' becomes power * (inv_pi / area) (AreaLight.cpp:170-179), with the area the
    representation's own: plane |x*y|, sphere 1.6075-ellipsoid, mesh area * bbox scale."""
    pw = {"power": [10, 10, 10]}
    sc = ignis_amd.Scene.from_string(_emitter_doc({"type": "rectangle", "width": 2, "height": 3}, pw))
    assert sc.desc.lights[0].radiance[0] == pytest.approx(10 / (np.pi * 6), rel=1e-5)
    sc = ignis_amd.Scene.from_string(_emitter_doc({"type": "sphere", "radius": 2}, pw))
    assert sc.desc.lights[0].radiance[1] == pytest.approx(10 / (np.pi * _ellipsoid_area(2, 2, 2, 1.6075)), rel=1e-5)
    # unit cube scaled by 2 along x: area 6 * scale (w h + w d + h d) / half_area = 6 * 5 / 3
    sc = ignis_amd.Scene.from_string(_emitter_doc({"type": "cube", "width": 1, "height": 1, "depth": 1}, pw,
                                                  transform=[{"scale": [2, 1, 1]}]))
    assert sc.desc.lights[0].type == _native.LIGHT_MESH
    assert sc.desc.lights[0].radiance[2] == pytest.approx(10 / (np.pi * 10), rel=1e-4)


def test_principled_parameters():
    """PrincipledBSDF::serialize (PrincipledBSDF.cpp:11-60): defaults, ior table, and
    principled::compute_roughness (roughness^2, anisotropic aspect sqrt(1 - 0.9 a))."""
    doc = {"bsdfs": [{"type": "principled", "name": "a"},
                     {"type": "principled", "name": "b", "roughness": 0.6, "anisotropic": 0.5, "metallic": 0.3,
                      "ior_material": "water", "thin": True, "clearcoat_top_only": False, "sheen": 0.25},
                     {"type": "principled", "name": "c", "roughness_u": 0.2, "roughness_v": 0.05, "ior": 1.33}],
           "shapes": [{"type": "rectangle", "name": "r"}],
           "entities": [{"name": "e%d" % i, "shape": "r", "bsdf": n} for i, n in enumerate("abc")]}
    sc = ignis_amd.Scene.from_string(doc)
    d = sc.desc
    mats = [d.materials[d.entities[i].material] for i in range(3)]
    a, b, c = mats
    assert a.bsdf_type == 4
    np.testing.assert_allclose(a.kd[:], [0.8, 0.8, 0.8])
    assert a.ior == pytest.approx(1.5046)
    assert (a.alpha_u, a.alpha_v) == (pytest.approx(0.25), pytest.approx(0.25))
    assert a.clearcoat_roughness == pytest.approx(0.1) and a.clearcoat_top_only == 1 and a.thin == 0
    aspect = np.sqrt(1 - 0.5 * 0.9)
    assert b.alpha_u == pytest.approx(0.36 / aspect, rel=1e-6) and b.alpha_v == pytest.approx(0.36 * aspect, rel=1e-6)
    assert b.ior == pytest.approx(1.333) and b.metallic == pytest.approx(0.3) and b.sheen == pytest.approx(0.25)
    assert b.thin == 1 and b.clearcoat_top_only == 0
    assert (c.alpha_u, c.alpha_v, c.ior) == (pytest.approx(0.2), pytest.approx(0.05), pytest.approx(1.33))


def test_procedural_geometry_matches_frozen_fixture():
    """Every procedural shape the scenes use, and the plane / sphere emitter
    detection on the scene meshes, reproduce tests/golden/procedural_shapes.npz
    bit for bit (tests/golden/make_shape_fixture.py)."""
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    import make_shape_fixture

    ref = np.load(os.path.join(os.path.dirname(__file__), "golden", "procedural_shapes.npz"))
    got = make_shape_fixture.generate()
    assert sorted(got) == sorted(ref.files)
    for k in ref.files:
        np.testing.assert_array_equal(got[k], ref[k], err_msg=k)
