"""Copy the BASELINE scene data out of the reference checkout into scenes/.

Runs in the build container only (the GPU box has no /root/reference).  The
scene JSON files are re-serialised (externals merged, so primitives.json is
self-contained) and the PLY meshes they reference are copied byte for byte.
These are data fixtures -- scene descriptions and triangle meshes -- not
reference source code.

Sources (relative to /root/reference):
  scenes/diamond_scene.json, scenes/meshes/{Bottom,Top,Left,Right,Back,Diamond}.ply
  scenes/primitives.json + scenes/primitives_data.json
"""
import json
import os
import shutil
import sys

REF = "/root/reference/scenes"
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
OUT = os.path.join(ROOT, "scenes")


def load(name):
    with open(os.path.join(REF, name)) as f:
        return json.load(f)


def merge_externals(doc):
    for ext in doc.pop("externals", []):
        sub = load(ext["filename"])
        for k, v in sub.items():
            if k in doc and isinstance(doc[k], list):
                doc[k] = doc[k] + v
            else:
                doc.setdefault(k, v)
    return doc


def main():
    if not os.path.isdir(REF):
        print("reference scenes not available; nothing to do", file=sys.stderr)
        return 1
    os.makedirs(os.path.join(OUT, "meshes"), exist_ok=True)
    for name in ["diamond_scene.json", "primitives.json"]:
        doc = merge_externals(load(name))
        with open(os.path.join(OUT, name), "w") as f:
            json.dump(doc, f, indent=1, sort_keys=True)
            f.write("\n")
        for shape in doc.get("shapes", []):
            fn = shape.get("filename")
            if fn:
                dst = os.path.join(OUT, fn)
                os.makedirs(os.path.dirname(dst), exist_ok=True)
                shutil.copyfile(os.path.join(REF, fn), dst)
    print("wrote", OUT)
    return 0


if __name__ == "__main__":
    sys.exit(main())
