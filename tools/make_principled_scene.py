"""Writes scenes/principled.json: a 3x3 grid of principled-BSDF spheres
(bsdf/principled.art) covering its lobes -- diffuse + specular, metallic,
sheen, clearcoat (top only and both sides), specular transmission, thin with
diffuse transmission and flatness, anisotropic roughness, specular tint --
on a diffuse ground under a plane area light and a dim environment."""
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

VARIANTS = [
    ("p_default", {}),
    ("p_metal", {"base_color": [0.9, 0.6, 0.3], "metallic": 1.0, "roughness": 0.3}),
    ("p_sheen", {"base_color": [0.3, 0.5, 0.9], "sheen": 1.0, "sheen_tint": 0.5, "roughness": 0.8}),
    ("p_clearcoat", {"base_color": [0.8, 0.1, 0.1], "clearcoat": 1.0, "clearcoat_gloss": 0.7, "roughness": 0.6}),
    ("p_clearcoat_both", {"base_color": [0.1, 0.6, 0.2], "clearcoat": 0.8, "clearcoat_top_only": False,
                          "clearcoat_roughness": 0.3}),
    ("p_glass", {"base_color": [0.95, 0.95, 1.0], "specular_transmission": 1.0, "roughness": 0.15, "ior": 1.45}),
    ("p_thin", {"base_color": [0.9, 0.8, 0.5], "thin": True, "diffuse_transmission": 0.6, "flatness": 0.5,
                "specular_transmission": 0.3, "roughness": 0.4}),
    ("p_aniso", {"base_color": [0.7, 0.7, 0.7], "metallic": 0.7, "roughness": 0.5, "anisotropic": 0.8}),
    ("p_tint", {"base_color": [0.2, 0.9, 0.6], "specular_tint": 1.0, "roughness_u": 0.2, "roughness_v": 0.05,
                "ior_material": "water"}),
]


def scene():
    bsdfs = [{"type": "diffuse", "name": "ground", "reflectance": [0.7, 0.7, 0.7]},
             {"type": "diffuse", "name": "black", "reflectance": [0, 0, 0]}]
    ents = [{"name": "ground", "shape": "ground", "bsdf": "ground"},
            {"name": "Light", "shape": "lightquad", "bsdf": "black"}]
    for k, (name, params) in enumerate(VARIANTS):
        bsdfs.append(dict({"type": "principled", "name": name}, **params))
        x, y = (k % 3 - 1) * 1.2, (k // 3 - 1) * 1.2
        ents.append({"name": "s_" + name, "shape": "ball", "bsdf": name,
                     "transform": [{"translate": [x, y, 0.45]}]})
    return {
        "technique": {"type": "path", "max_depth": 16},
        "camera": {"type": "perspective", "fov": 45, "near_clip": 0.01, "far_clip": 100,
                   "transform": [{"lookat": {"origin": [0, -4.5, 3.2], "target": [0, 0, 0.3], "up": [0, 0, 1]}}]},
        "film": {"size": [512, 512]},
        "bsdfs": bsdfs,
        "shapes": [{"type": "rectangle", "name": "ground", "width": 12, "height": 12},
                   {"type": "icosphere", "name": "ball", "radius": 0.45, "subdivisions": 3},
                   {"type": "rectangle", "name": "lightquad", "flip_normals": True, "width": 3, "height": 3,
                    "transform": [{"translate": [0, 0, 4]}]}],
        "entities": ents,
        "lights": [{"type": "area", "name": "AreaLight", "entity": "Light", "radiance": [6, 6, 6]},
                   {"type": "env", "name": "env", "radiance": [0.3, 0.3, 0.35]}],
    }


if __name__ == "__main__":
    path = os.path.join(ROOT, "scenes", "principled.json")
    with open(path, "w") as f:
        json.dump(scene(), f, indent=1)
    print("wrote", path)
