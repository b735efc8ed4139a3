"""Expected image ratio of the cycles-box evaluation scene (tests/test_eval.py,
MODEL DIFFERENCE): the reference code's principled cube against the same cube
with Blender 3.4's Cycles principled diffuse lobe, integrated numerically.

The scene is one convex cube (principled: base colour 0.8, roughness 0.5, no
metal / sheen / clearcoat / transmission) under a point light and a constant
environment.  A convex object sees neither itself nor anything else, so the
radiance towards the camera is exactly

    L(x, wo) = f(wo, wl) cos_l I / d^2          (point light; unoccluded when cos_l > 0)
             + L_env * A(wo),  A(wo) = integral over the hemisphere of f(wo, wi) cos_i dwi

for every camera ray that hits the cube, and L_env for the rest.  f is the
principled BSDF as the oracle restates it (bsdf/principled.art;
oracle_principled_eval, TEST INFRASTRUCTURE), evaluated with three diffuse lobes:

  model 0  the reference's evalDiffuseTerm (principled.art:117-129): Disney
           2015's split with the retro-reflection weight
           R = (1 + |cos theta_vl|) * (alpha_u + alpha_v) / 2 on alpha = roughness^2;
  model 1  Blender 3.x Cycles (bsdf_principled_diffuse, the PLY was written by
           Blender 3.4.0): the same split with R = roughness * (1 + cos theta_vl)
           on the roughness input itself;
  model 2  Burley 2012 (F_D90 = 0.5 + 2 roughness cos^2 theta_d), for comparison.

The specular lobe, the lights and the camera are the same in all three, so the
ratio of the cube's mean radiance under model 0 and model 1 is the expected
ratio of the reference code's image to Cycles' image, as far as the diffuse
models are the difference.  A(wo) depends on the angle of wo to the normal only
(isotropic BSDF): tabulated on 1024 cosines, each a Gauss-Legendre (cos theta)
x uniform (phi) quadrature; pixels average a 4x4 grid of camera rays, as
tests/test_eval.py's pixel_coverage casts them.  Hits come from the oracle's
trace_hits.  The cube mask is the test's: reference pixels brighter than the
0.0509 environment.

Writes tests/golden/cycles_box_model.json.  Run from the repository root:
    python tests/golden/cycles_box_model.py
"""
import ctypes as C
import json
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (os.path.join(ROOT, "ignis-masterthesis_amd"), ROOT, os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

import evalref as E  # noqa: E402
import ignis_amd  # noqa: E402
from oracle import oracle_py as O  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "cycles_box_model.json")


def principled_eval(mat, wo, wi, model):
    """f(wo, wi) * cos(wi) in a front-facing local frame (normal +z), n x 3 arrays."""
    L = O.lib()
    L.oracle_principled_eval.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_float), C.POINTER(C.c_float), C.c_int,
                                         C.POINTER(C.c_float)]
    wo = np.ascontiguousarray(wo, np.float32)
    wi = np.ascontiguousarray(wi, np.float32)
    out = np.zeros_like(wo)
    fp = lambda a: a.ctypes.data_as(C.POINTER(C.c_float))
    L.oracle_principled_eval(C.addressof(mat), len(wo), fp(wo), fp(wi), model, fp(out))
    return out


def albedo_table(mat, model, n_cos=1024, n_theta=96, n_phi=192):
    """A(cos_o) on n_cos cosines in (0, 1]: hemisphere quadrature of f cos."""
    x, wq = np.polynomial.legendre.leggauss(n_theta)
    ci = 0.5 * (x + 1)                      # cos theta_i in (0, 1)
    wc = 0.5 * wq                           # d(cos theta)
    phi = (np.arange(n_phi) + 0.5) * (2 * math.pi / n_phi)
    si = np.sqrt(np.maximum(0, 1 - ci * ci))
    wi = np.stack([np.outer(si, np.cos(phi)), np.outer(si, np.sin(phi)), np.repeat(ci[:, None], n_phi, 1)], -1).reshape(-1, 3)
    wgt = np.repeat(wc[:, None], n_phi, 1).reshape(-1) * (2 * math.pi / n_phi)
    cos_o = (np.arange(n_cos) + 0.5) / n_cos
    table = np.zeros((n_cos, 3))
    for k, co in enumerate(cos_o):
        wo = np.tile([math.sqrt(max(0.0, 1 - co * co)), 0.0, co], (len(wi), 1))
        table[k] = (principled_eval(mat, wo, wi, model) * wgt[:, None]).sum(0)
    return cos_o, table


def pixel_rays(sc, jx, jy, grid):
    w, h = sc.film_size
    c = sc.desc.camera
    eye, dr, up = np.array(c.eye[:]), np.array(c.dir[:]), np.array(c.up[:])
    right = np.cross(dr, up)
    right /= np.linalg.norm(right)
    aspect = c.aspect if c.aspect > 0 else w / h
    sx, sy = (math.tan(c.fov / 2) * aspect, math.tan(c.fov / 2)) if c.vertical_fov else (math.tan(c.fov / 2), math.tan(c.fov / 2) / aspect)
    ys, xs = np.mgrid[0:h, 0:w]
    nx = 2 * (xs + (jx + 0.5) / grid) / w - 1
    ny = 1 - 2 * (ys + (jy + 0.5) / grid) / h
    v = sx * nx[..., None] * right + sy * ny[..., None] * up + dr
    v /= np.linalg.norm(v, axis=-1, keepdims=True)
    rays = np.zeros((w * h, 8), np.float32)
    rays[:, 0:3] = eye
    rays[:, 3:6] = v.reshape(-1, 3)
    rays[:, 6], rays[:, 7] = c.near_clip, c.far_clip
    return rays


def model_images(grid=4, models=(0, 1, 2), quad=(96, 192)):
    sc = ignis_amd.Scene.from_file(E.scene_path("cycles-box"))
    d = sc.desc
    assert d.num_entities == 1 and d.num_materials == 1 and d.materials[0].bsdf_type == 4
    mat = d.materials[0]
    lights = [d.lights[i] for i in range(d.num_lights)]
    point = [L for L in lights if L.type == ignis_amd._native.LIGHT_POINT]
    env = [L for L in lights if L.type == ignis_amd._native.LIGHT_ENV]
    assert len(point) == 1 and len(env) == 1
    lpos, lint = np.array(point[0].origin[:]), np.array(point[0].radiance[:])
    lenv = np.array(env[0].radiance[:])
    # the cube's world-space face normals (flat faces: its vertex normals are the face normals)
    en = d.entities[0]
    m = d.meshes[d.shapes[en.shape].mesh]
    V = np.ctypeslib.as_array(m.vertices, (m.num_vertices * 3,)).reshape(-1, 3).astype(np.float64)
    F = np.ctypeslib.as_array(m.indices, (m.num_faces * 3,)).reshape(-1, 3)
    T = np.array(en.to_global[:]).reshape(3, 4)
    Vw = V @ T[:, :3].T + T[:, 3]
    fn = np.cross(Vw[F[:, 1]] - Vw[F[:, 0]], Vw[F[:, 2]] - Vw[F[:, 0]])
    fn /= np.linalg.norm(fn, axis=1, keepdims=True)
    orc = O.OracleScene(sc)
    tables = {mo: albedo_table(mat, mo, n_theta=quad[0], n_phi=quad[1]) for mo in models}
    w, h = sc.film_size
    imgs = {mo: np.zeros((h * w, 3)) for mo in models}
    for jy in range(grid):
        for jx in range(grid):
            rays = pixel_rays(sc, jx, jy, grid)
            ep, tuv = orc.trace_hits(rays, 1)
            hit = ep[:, 0] >= 0
            x = rays[hit, :3].astype(np.float64) + tuv[hit, :1] * rays[hit, 3:6]
            n = fn[ep[hit, 1]]
            n = np.where((n * rays[hit, 3:6]).sum(1, keepdims=True) > 0, -n, n)  # the side the ray sees
            # local frame (t, b, n)
            a = np.where(np.abs(n[:, :1]) > 0.9, [[0, 1, 0]], [[1, 0, 0]])
            t = np.cross(a, n)
            t /= np.linalg.norm(t, axis=1, keepdims=True)
            b = np.cross(n, t)
            to_local = lambda v: np.stack([(v * t).sum(1), (v * b).sum(1), (v * n).sum(1)], 1)
            wo = to_local(-rays[hit, 3:6].astype(np.float64))
            dl = lpos - x
            d2 = (dl * dl).sum(1)
            wl = to_local(dl / np.sqrt(d2)[:, None])
            lit = wl[:, 2] > 0
            for mo in models:
                cos_o, tab = tables[mo]
                env_term = np.stack([np.interp(wo[:, 2], cos_o, tab[:, c]) for c in range(3)], 1) * lenv
                fl = principled_eval(mat, wo, wl, mo).astype(np.float64)
                pt = np.where(lit[:, None], fl * lint / d2[:, None], 0)
                img = imgs[mo]
                img[hit] += env_term + pt
                img[~hit] += lenv
    return {mo: (img / grid ** 2).reshape(h, w, 3) for mo, img in imgs.items()}


def main():
    imgs = model_images()
    ref = E.reference_image("cycles-box")
    cube = ref.mean(axis=2) > 0.06
    mean = {mo: float(img[cube].mean()) for mo, img in imgs.items()}
    # quadrature convergence: the same with half the nodes per axis
    half = model_images(grid=2, models=(0, 1), quad=(48, 96))
    out = {
        "scene": "scenes/evaluation/cycles-box.json",
        "cube_pixels": int(cube.sum()),
        "mean_cube_radiance": {"reference_model": mean[0], "cycles_disney2015_on_roughness": mean[1],
                               "burley2012": mean[2], "cycles_reference_image": float(ref[cube].mean())},
        "expected_ratio": mean[0] / mean[1],
        "expected_ratio_vs_burley2012": mean[0] / mean[2],
        "expected_ratio_coarse": float(half[0][cube].mean() / half[1][cube].mean()),
        "background_radiance": float(imgs[0][~cube].mean()),
        "note": "reference code / Cycles (Blender 3.x principled diffuse), cube mask = reference pixels > 0.06; "
                "tests/golden/cycles_box_model.py",
    }
    with open(OUT, "w") as f:
        json.dump(out, f, indent=1)
    np.save(os.path.join(os.path.dirname(OUT), "cycles_box_model_ref.npy"), imgs[0].astype(np.float32)) if os.environ.get("SAVE_IMG") else None
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
