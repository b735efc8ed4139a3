"""The SceneDatabase seam: the reference's table layouts, written
by tests/refdb.py from a scene igx's JSON loader read, go through
igx_scene_from_database and must give back the same igx_scene_desc, field by
field (CPU, no GPU).  Malformed tables are refused with a message.  The GPU
twin (tests/test_gpu.py::test_database_adapter_renders_bit_identically)
renders both descs."""
import ctypes as C
import os

import numpy as np
import pytest

from refdb import RefDatabase

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

import ignis_amd  # noqa: E402
from ignis_amd import _native as N  # noqa: E402

SCENES = ["diamond_scene.json", "primitives.json", "materials.json", "principled.json",
          "evaluation/cbox-d6.json", "evaluation/sphere-light-ico.json", "evaluation/multilight-uniform.json"]


def _struct_eq(a, b, path, skip=()):
    for name, typ in a._fields_:
        if name in skip:
            continue
        x, y = getattr(a, name), getattr(b, name)
        if isinstance(x, C.Structure):
            _struct_eq(x, y, f"{path}.{name}", skip)
        elif isinstance(x, C.Array):
            xa, ya = np.array(list(x)), np.array(list(y))
            assert np.array_equal(xa.view(np.uint32) if xa.dtype == np.float32 else xa,
                                  ya.view(np.uint32) if ya.dtype == np.float32 else ya), f"{path}.{name}: {xa} != {ya}"
        elif not hasattr(x, "contents") and not isinstance(x, (int, float)) and x is not None:
            continue
        elif isinstance(x, float):
            assert np.float32(x).view(np.uint32) == np.float32(y).view(np.uint32), f"{path}.{name}: {x} != {y}"
        elif isinstance(x, int) or x is None:
            assert x == y, f"{path}.{name}: {x} != {y}"


def _arr(ptr, n, dt):
    return np.ctypeslib.as_array(ptr, (n,)).astype(dt) if n else np.zeros(0, dt)


def assert_desc_equal(d1, d2):
    for k in ("film_width", "film_height", "num_meshes", "num_shapes", "num_entities", "num_materials", "num_lights"):
        assert getattr(d1, k) == getattr(d2, k), k
    _struct_eq(d1.camera, d2.camera, "camera")
    _struct_eq(d1.technique, d2.technique, "technique")
    assert list(d1.scene_bbox_min) == list(d2.scene_bbox_min) and list(d1.scene_bbox_max) == list(d2.scene_bbox_max)
    for i in range(d1.num_meshes):
        m1, m2 = d1.meshes[i], d2.meshes[i]
        assert (m1.num_vertices, m1.num_faces) == (m2.num_vertices, m2.num_faces)
        nv, nf = m1.num_vertices, m1.num_faces
        for f, n, dt in (("vertices", 3 * nv, np.float32), ("normals", 3 * nv, np.float32),
                         ("texcoords", 2 * nv, np.float32), ("indices", 3 * nf, np.uint32)):
            a, b = _arr(getattr(m1, f), n, dt), _arr(getattr(m2, f), n, dt)
            assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), f"mesh {i} {f}"
    for i in range(d1.num_shapes):
        _struct_eq(d1.shapes[i], d2.shapes[i], f"shape[{i}]", skip=("ref_bvh", "ref_bvh_bytes"))
    for i in range(d1.num_entities):
        _struct_eq(d1.entities[i], d2.entities[i], f"entity[{i}]")
    for i in range(d1.num_materials):
        _struct_eq(d1.materials[i], d2.materials[i], f"material[{i}]")
    for i in range(d1.num_lights):
        _struct_eq(d1.lights[i], d2.lights[i], f"light[{i}]")


@pytest.mark.parametrize("name", SCENES)
def test_adapter_gives_back_the_loader_desc(name):
    scene = ignis_amd.Scene.from_file(os.path.join(ROOT, "scenes", name))
    ref = RefDatabase(scene)
    db, sv, keep = ref.views()
    back = ignis_amd.Scene.from_database(db, sv)
    d1, d2 = scene.desc, back.desc
    assert_desc_equal(d1, d2)
    # every trimesh shape carries its reference BLAS blob, byte for byte
    for i in range(d2.num_shapes):
        s = d2.shapes[i]
        if s.type == 0:
            assert s.ref_bvh and s.ref_bvh_bytes > 16
            hdr = np.frombuffer(C.string_at(s.ref_bvh, 16), np.uint32)
            assert s.ref_bvh_bytes == 16 + 64 * hdr[0] + 48 * hdr[1]
        else:
            assert not s.ref_bvh


def test_adapter_without_blas_tables():
    scene = ignis_amd.Scene.from_file(os.path.join(ROOT, "scenes", "diamond_scene.json"))
    db, sv, keep = RefDatabase(scene, with_blas=False).views()
    back = ignis_amd.Scene.from_database(db, sv)
    assert_desc_equal(scene.desc, back.desc)
    assert all(not back.desc.shapes[i].ref_bvh for i in range(back.desc.num_shapes))


def test_record_offsets_follow_the_reference_padding():
    """DynTable::addLookup pads by a full 16 B when already aligned (DynTable.h:20-23):
    the first record sits at 0, later ones never directly after an aligned end."""
    scene = ignis_amd.Scene.from_file(os.path.join(ROOT, "scenes", "primitives.json"))
    ref = RefDatabase(scene)
    offs = [o for _, _, o in ref.shapes.lookups]
    assert offs[0] == 0 and all(o % 16 == 0 for o in offs)
    assert all(b - a > 0 for a, b in zip(offs, offs[1:]))


def _corrupt(mutate, match):
    scene = ignis_amd.Scene.from_file(os.path.join(ROOT, "scenes", "primitives.json"))
    ref = RefDatabase(scene)
    mutate(ref)
    db, sv, keep = ref.views()
    with pytest.raises(ignis_amd.IgxError, match=match):
        ignis_amd.Scene.from_database(db, sv)


def test_malformed_tables_are_refused():
    def bad_type(r):
        t, f, o = r.shapes.lookups[0]
        r.shapes.lookups[0] = (77, f, o)
    _corrupt(bad_type, "provider type")

    def truncated(r):
        r.shapes.data = r.shapes.data[:-8]
    _corrupt(truncated, "beyond the end")

    def entity_shape(r):
        rec = np.frombuffer(bytes(r.entities.data[:144]), np.uint32).copy()
        rec[33] = 999
        r.entities.data[:144] = rec.tobytes()
    _corrupt(entity_shape, "shape id")

    def entity_material(r):
        rec = np.frombuffer(bytes(r.entities.data[:144]), np.uint32).copy()
        rec[34] = 999
        r.entities.data[:144] = rec.tobytes()
    _corrupt(entity_material, "material id")

    def leaf_entity(r):
        rec = np.frombuffer(bytes(r.leaves[:96]), np.uint32).copy()
        rec[3] = 5000
        r.leaves[:96] = rec.tobytes()
    _corrupt(leaf_entity, "entity id")

    def short_blas(r):
        r.primbvh.data = r.primbvh.data[:40]
    _corrupt(short_blas, "beyond the end")

    def huge_blas_offset(r):
        # user2 (high word of the BLAS offset in floats) with bit 30 set: offset * 4
        # wraps to the low word's bytes unless the offset is checked first
        recs = np.frombuffer(bytes(r.leaves), np.uint32).copy().reshape(-1, 24)
        recs[:, 23] |= 0x40000000
        r.leaves[:] = recs.tobytes()
    _corrupt(huge_blas_offset, "BLAS offset beyond the table")


def test_corrupted_transform_is_seen():
    """A changed toGlobal column in the entity table shows up in the desc (the
    adapter reads the table, it does not re-derive it)."""
    scene = ignis_amd.Scene.from_file(os.path.join(ROOT, "scenes", "diamond_scene.json"))
    ref = RefDatabase(scene)
    rec = np.frombuffer(bytes(ref.entities.data[144:288]), np.float32).copy()
    rec[12 + 9] += 0.25  # toGlobal translation x of entity 1 (column 3, row 0)
    ref.entities.data[144:288] = rec.tobytes()
    db, sv, keep = ref.views()
    back = ignis_amd.Scene.from_database(db, sv)
    with pytest.raises(AssertionError, match=r"entity\[1\]\.to_global"):
        assert_desc_equal(scene.desc, back.desc)


def test_cpp_database_roundtrip(tmp_path):
    """The C++ side of the seam (host/scene_database.h, host/Device.h): igx's
    loader writes the reference's tables (serialize_scene), the facade's view
    of them goes through igx_scene_from_database, and the loader's desc comes
    back bit for bit with a readable BLAS blob per trimesh shape
    (tests/native/db_roundtrip.cpp, g++ against libigx.so, no GPU call)."""
    import subprocess

    pkg = os.path.join(ROOT, "ignis-masterthesis_amd")
    exe = str(tmp_path / "db_roundtrip")
    subprocess.run(["g++", "-O1", "-std=c++17", "-I", os.path.join(ROOT, "include"), "-I", os.path.join(pkg, "host"),
                    os.path.join(ROOT, "tests", "native", "db_roundtrip.cpp"), "-o", exe, "-L", pkg, "-ligx",
                    f"-Wl,-rpath,{pkg}", "-L/opt/rocm/lib", "-lamdhip64"], check=True)
    scenes = [os.path.join(ROOT, "scenes", s) for s in SCENES]
    out = subprocess.run([exe] + scenes, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0 and out.stdout.strip().endswith("ok"), out.stdout + out.stderr


def test_scene_names_for_bindings():
    """igx_scene_find_material / igx_scene_entity_name: the lookups a binding
    uses to re-index igx's shading tables by the reference loader's ids."""
    L = N.lib()
    scene = ignis_amd.Scene.from_file(os.path.join(ROOT, "scenes", "diamond_scene.json"))
    d = scene.desc
    names = [L.igx_scene_entity_name(scene._h, i).decode() for i in range(d.num_entities)]
    assert sorted(names) == sorted(["AreaLight", "Bottom", "Top", "Left", "Right", "Back", "Diamond1", "Diamond2", "Diamond3"])
    assert L.igx_scene_entity_name(scene._h, d.num_entities) is None
    light_mat = L.igx_scene_find_material(scene._h, b"mat-Light", b"AreaLight")
    diamond = L.igx_scene_find_material(scene._h, b"mat-Diamond", None)
    assert light_mat >= 0 and d.materials[light_mat].light == 0
    assert diamond >= 0 and d.materials[diamond].bsdf_type == 1
    assert L.igx_scene_find_material(scene._h, b"mat-Light", None) == -1  # the emissive one is its own material
    assert L.igx_scene_find_material(scene._h, b"nope", None) == -1
    for i in range(d.num_entities):
        if names[i].startswith("Diamond"):
            assert d.entities[i].material == diamond
