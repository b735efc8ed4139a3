"""igx's C++ scene loader against an independent restatement of the reference's
scene loading (tests/scene_ref.py), field by field, on every scene the parity
tests render.  A corrupted descriptor field must be caught."""
import ctypes as C
import glob
import os

import pytest

import ignis_amd
import scene_ref

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def scene_files():
    files = [os.path.join(ROOT, "scenes", f) for f in ("diamond_scene.json", "primitives.json", "materials.json",
                                                       "principled.json")]
    for f in sorted(glob.glob(os.path.join(ROOT, "scenes", "evaluation", "*.json"))):
        if f.endswith("-base.json") or f.endswith("references.json"):
            continue
        files.append(f)
    return files


@pytest.mark.parametrize("path", scene_files(), ids=os.path.basename)
def test_loader_matches_reference_reading(path):
    try:
        sc = ignis_amd.Scene.from_file(path)
    except ignis_amd.IgxError as e:
        pytest.skip(f"not loadable by igx: {e}")
    scene_ref.check_desc(path, sc.desc)


@pytest.mark.parametrize("field", ["camera.eye", "entity.to_global", "light.x_axis", "material.kd", "light.normal"])
def test_corrupted_descriptor_field_is_caught(field):
    path = os.path.join(ROOT, "scenes", "diamond_scene.json")
    sc = ignis_amd.Scene.from_file(path)
    d = sc.desc
    scene_ref.check_desc(path, d)  # clean
    if field == "camera.eye":
        d.camera.eye[1] += 0.01
    elif field == "entity.to_global":
        d.entities[2].to_global[3] += 0.05
    elif field == "light.x_axis":
        d.lights[0].x_axis[0] *= 1.01
    elif field == "material.kd":
        d.materials[d.entities[1].material].kd[1] = 0.5
    elif field == "light.normal":
        for k in range(3):
            d.lights[0].normal[k] = -d.lights[0].normal[k]
    with pytest.raises(AssertionError):
        scene_ref.check_desc(path, d)
