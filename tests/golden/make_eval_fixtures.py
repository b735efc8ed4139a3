"""Copy the reference's evaluation scenes and their converged reference images
into scenes/evaluation/ (data fixtures: scene descriptions, meshes, EXR images).

Runs in the build container only (the GPU box has no /root/reference).  Files
are copied byte for byte with their relative layout kept, so the scenes'
`externals` and `../meshes/*.ply` paths resolve the same way they do in the
reference checkout.  The reference image of a scene is picked exactly as
`scripts/RunEvaluations.py:get_reference_path` (lines 18-38) picks it: the
shortest `ref-<stem>*.exr`, dropping up to two trailing `-section`s of the stem.

The scene list is every `scenes/evaluation/*.json` (minus `-base` files, as
RunEvaluations.py does) that igx's loader accepts; see tests/test_eval.py.
"""
import glob
import json
import os
import shutil
import sys

REF = "/root/reference/scenes"
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
OUT = os.path.join(ROOT, "scenes")

SCENES = [
    "cbox-d1", "cbox-d6", "emissive-plane", "emissive-plane-nopt", "emissive-plane-scale",
    "emissive-plane-scale-nopt", "flipped-prim-diffuse", "flipped-prim-glass",
    "multilight", "multilight-uniform", "multilight-simple", "multilight-hierarchy",
    "plane-d1", "plane-d6", "point", "room",
    "sphere-light-ico", "sphere-light-ico-nopt", "sphere-light-pure", "sphere-light-uv",
    "three-planes-dielectric", "three-planes-glass", "three-planes-interface",
    "two-planes-mirror", "two-planes-plastic",
    # Blender Cycles references: principled BSDF + point (power) + constant environment;
    # principled cone + sun light over a checker-textured diffuse ground
    "cycles-box", "cycles-sun",
]


def reference_image(stem, ref_dir):
    """RunEvaluations.py:18-38."""
    base = stem
    for _ in range(3):
        found = glob.glob(os.path.join(ref_dir, f"ref-{base}*.exr"))
        if found:
            return min(found, key=len)
        base = base[:base.rfind("-")]
    return None


def deps(path, seen):
    """The scene file, its externals (recursively) and the mesh files it names."""
    if path in seen:
        return
    seen.add(path)
    with open(path) as f:
        doc = json.load(f)
    d = os.path.dirname(path)
    for ext in doc.get("externals", []):
        deps(os.path.normpath(os.path.join(d, ext["filename"])), seen)
    for shape in doc.get("shapes", []):
        fn = shape.get("filename")
        if fn:
            seen.add(os.path.normpath(os.path.join(d, fn)))


def main():
    if not os.path.isdir(REF):
        print("reference scenes not available; nothing to do", file=sys.stderr)
        return 1
    files = set()
    refs = {}
    for stem in SCENES:
        deps(os.path.join(REF, "evaluation", stem + ".json"), files)
        img = reference_image(stem, os.path.join(REF, "evaluation", "references"))
        assert img, stem
        files.add(img)
        refs[stem] = os.path.relpath(img, REF)
    for src in sorted(files):
        dst = os.path.join(OUT, os.path.relpath(src, REF))
        os.makedirs(os.path.dirname(dst), exist_ok=True)
        shutil.copyfile(src, dst)
    with open(os.path.join(OUT, "evaluation", "references.json"), "w") as f:
        json.dump(refs, f, indent=1, sort_keys=True)
        f.write("\n")
    print(f"copied {len(files)} files into {OUT}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
