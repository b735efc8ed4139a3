"""Image parity against the reference's own converged images
(scenes/evaluation/references/*.exr) with the reference's own metric and
tolerances (scripts/RunEvaluations.py, restated in tests/evalref.py).

The reference images were rendered by Mitsuba 2/3 (`-4096` files) or Radiance
(`-rad` files), not by Ignis; RunEvaluations.py compares Ignis' GPU and CPU
devices against them at 1024 spp.  The scenes fall into three groups:

* DIRECT: the reference code's semantics agree with the other renderer's, so
  the HIP device must pass RunEvaluations' check as is (err < predef_eps at
  1024 spp).
* TRANSFORMED: the reference code at this commit renders a different (but
  derivable) image; the test checks the HIP device against the reference image
  transformed by the exact relation the reference code implies:
  - plane-d6: the Lambert BSDF is evaluated two-sided (`absolute_cos`,
    bsdf/diffuse.art:3) and the NEE shadow ray toward the back hemisphere of
    the open floor quad is unoccluded, so the constant environment lights the
    floor from below as much as from above: floor radiance doubles.  With the
    d1 image (environment coverage only) this is exactly
    expected = 2 * ref_d6 - ref_d1.
  - multilight-*: the same back-side NEE of the 0.2 constant environment adds
    0.2 * kd on the floor quad: expected = ref + 0.2 * kd * coverage, the floor
    coverage of each pixel measured by casting the camera's jittered rays.
  - cbox-d6: the luminaire carries a 0.94-albedo diffuse BSDF, and a hit point
    on it (org + t*dir, shapes/trimesh.art:31) lands a rounding error below or
    above the emitter plane.  NEE from a point just below sees the emitter's
    front over almost a hemisphere (spherical-rectangle sampling,
    light/area.art:116-195; cosine sign taken from the receiver's side,
    light/area.art:17; shadow ray ending at 1 - offset, pathtracer.art:103),
    so the luminaire reflects ~kd*L of its own light and acts as a ~16 %
    brighter source for the whole box; BSDF-sampled rays cannot reproduce it,
    so NEE-off renders match Mitsuba.  With a black luminaire BSDF (its
    reflected light is ~1 % of its emission in Mitsuba's image) the render must
    pass the unmodified reference image.
  - flipped-prim-diffuse: a mirroring entity transform turns the triangle
    face normal (computed from the transformed vertices, shapes/trimesh.art:21-24)
    inward while the vertex-normal shading frame stays outward, so the shading
    frame faces into the cylinder.  The scene is symmetric under z -> -z, so
    the cylinder without the mirror must render the reference image mirrored
    vertically.
* MODEL DIFFERENCE: cycles-box is Blender Cycles' image of a principled cube
  (roughness 0.5, no metal / sheen / clearcoat) under a point light (given
  by `power`) and a constant environment.  principled.art's diffuse lobe is
  Disney 2015's split (bsdf/principled.art:112-124) with its retro-reflection
  weight rr = (1 + cos theta_vl) * (alpha_u + alpha_v) / 2 taken on the
  squared roughness (alpha = 0.25), where Cycles' principled diffuse is
  Burley 2012's with F_D90 = 0.5 + 2 roughness cos^2 theta_d on the roughness
  itself (0.5).  tests/golden/cycles_box_model.py integrates the convex cube
  under both lobes (point light + environment, no interreflection): the
  Cycles-model cube reproduces Cycles' image to 0.04 %, and the reference
  model's cube is 0.9558 of it.  The environment-only pixels must pass
  RunEvaluations' default eps as is, the cube's mean ratio must equal 0.9558
  within 0.5 %, and the whole image stays within twice the default eps.
* NOT COMPARABLE (not tested here): three-planes-* are
  Radiance images of caustics through glass from a 1 cm sphere light, which a
  path tracer whose shadow rays stop at glass (the reference's) only reaches by
  BSDF-sampling the tiny light.

CPU twins run the oracle on the DIRECT scenes at 128 spp, with the tolerance
scaled by 1024/128 (RelSE of an unbiased estimate falls as 1/spp).
"""
import json
import os
import sys

import numpy as np
import pytest

import evalref as E
import ignis_amd

DIRECT = [
    "cbox-d1", "emissive-plane", "emissive-plane-nopt", "emissive-plane-scale", "emissive-plane-scale-nopt",
    "flipped-prim-glass", "plane-d1", "point", "room", "sphere-light-ico", "sphere-light-ico-nopt",
    "sphere-light-pure", "sphere-light-uv", "two-planes-mirror", "two-planes-plastic",
    # Blender Cycles: sun light (light/sun.art), principled cone, checker-textured ground
    "cycles-sun",
]
MULTILIGHT = ["multilight", "multilight-uniform", "multilight-simple", "multilight-hierarchy"]
SPI = 8


def render_device(device, scene, spp, seed=0):
    w, h = scene.film_size
    device.upload(scene)
    device.set_option("capacity", 0)
    device.clear()
    p = ignis_amd.RenderParams()
    p.width, p.height, p.spi, p.seed = w, h, SPI, seed
    device.render_iterations(p, (spp + SPI - 1) // SPI)  # Runtime::step until SampleCount >= spp
    fb, it = device.framebuffer(w * h * 3)
    img, bad = E.sanitize(fb.reshape(h, w, 3) / it)
    return img, bad


def render_oracle(scene, spp, seed=0):
    from oracle import oracle_py as O

    w, h = scene.film_size
    fb, _ = O.OracleScene(scene).render(w, h, spp, seed=seed)
    return E.sanitize(fb.reshape(h, w, 3))


def load(stem):
    return ignis_amd.Scene.from_file(E.scene_path(stem))


def scene_from_doc(doc, base_dir):
    return ignis_amd.Scene.from_string(json.dumps(doc), base_dir)


def pixel_coverage(tracer, scene, entity_name_index, grid=8):
    """Fraction of each pixel whose jittered camera ray (uniform pixel sampler,
    sampler/pixel_sampler.art:4-10) first hits entity `entity_name_index`;
    `tracer` is the HIP device or the oracle (trace_hits)."""
    import math

    w, h = scene.film_size
    c = scene.desc.camera
    eye, dr, up = np.array(c.eye[:]), np.array(c.dir[:]), np.array(c.up[:])
    right = np.cross(dr, up)
    right /= np.linalg.norm(right)
    aspect = c.aspect if c.aspect > 0 else w / h  # compute_scale_from_{h,v}fov (camera/perspective.art:2-14)
    if c.vertical_fov:
        sy = math.tan(c.fov / 2)
        sx = sy * aspect
    else:
        sx = math.tan(c.fov / 2)
        sy = sx / aspect
    cov = np.zeros((h, w))
    for jy in range(grid):
        for jx in range(grid):
            ys, xs = np.mgrid[0:h, 0:w]
            nx = 2 * (xs + (jx + 0.5) / grid) / w - 1
            ny = 1 - 2 * (ys + (jy + 0.5) / grid) / h
            v = sx * nx[..., None] * right + sy * ny[..., None] * up + dr
            v /= np.linalg.norm(v, axis=-1, keepdims=True)
            rays = np.zeros((w * h, 8), np.float32)
            rays[:, 0:3] = eye
            rays[:, 3:6] = v.reshape(-1, 3)
            rays[:, 6], rays[:, 7] = c.near_clip, c.far_clip
            ep, _ = tracer.trace_hits(rays, 1)
            cov += (ep[:, 0] == entity_name_index).reshape(h, w)
    return cov / grid ** 2


# ------------------------------------------------------------------ CPU tests
def test_reference_images_decode():
    """Every committed reference image decodes (PIZ / ZIP EXR) to finite,
    non-negative RGB; alpha channels, where present, are exactly 1."""
    from exr_read import read_exr

    with open(os.path.join(E.EVAL_DIR, "references.json")) as f:
        paths = sorted(set(json.load(f).values()))
    assert len(paths) >= 15
    for rel in paths:
        img, attrs = read_exr(os.path.join(E.ROOT, "scenes", rel))
        assert attrs["compression"][1][0] in (3, 4)
        for ch in "RGB":
            assert img[ch].shape == (256, 256)
            assert np.isfinite(img[ch]).all() and (img[ch] >= 0).all(), rel
        if "A" in img:
            assert (img["A"] == 1).all(), rel
    # facts the scene files fix: plane-d1 shows the white environment (radiance
    # 1) wherever the floor is not in view, and the brightest Cornell-box pixels
    # are the luminaire's radiance (cbox-base.json)
    d1 = E.reference_image("plane-d1")
    assert np.abs(d1[:64] - 1).max() < 0.05 and abs(d1[:64].mean() - 1) < 1e-3
    c1 = E.reference_image("cbox-d1").reshape(-1, 3)
    lum = np.median(c1[c1[:, 0] > 15], axis=0)
    np.testing.assert_allclose(lum, [18.387, 10.9873, 2.75357], rtol=1e-2)


def test_error_image_metric():
    """RunEvaluations.py:80-87 on hand-made inputs."""
    ref = np.ones((10, 10, 3), np.float32)
    ref[0, 0] = 0
    img = ref * 1.1
    img[0, 0] = 0.5  # AbsSE pixel: 0.25, above the 99th percentile -> clamped
    err, _ = E.error_image(img, ref)
    # 297 values of 0.01 and 3 of 0.25 (R, G, B of the zero pixel); numpy's
    # linear 99th percentile sits at rank 296.01: 0.01 + 0.01 * 0.24
    p99 = 0.01 + 0.01 * 0.24
    assert err == pytest.approx((297 * 0.01 + 3 * p99) / 300, rel=1e-4)
    assert E.eps_for("room") == 1e-3 and E.eps_for("cbox-d6") == 5e-3 and E.eps_for("nosuch") == 1e-3


@pytest.mark.parametrize("stem", ["cbox-d1", "emissive-plane", "emissive-plane-scale", "flipped-prim-glass",
                                  "plane-d1", "point", "room", "sphere-light-pure", "sphere-light-uv",
                                  "two-planes-plastic", "cycles-sun"])
def test_oracle_matches_reference_image(stem):
    """CPU twin: the oracle (restated reference CPU device) at 128 spp against
    the reference image, eps scaled by 1024/128."""
    spp = 128
    img, bad = render_oracle(load(stem), spp)
    err, _ = E.error_image(img, E.reference_image(stem))
    assert bad == 0
    assert err < E.eps_for(stem) * (E.DEFAULT_SPP / spp), err


def test_oracle_plane_d6_two_sided_lambert():
    spp = 128
    img, _ = render_oracle(load("plane-d6"), spp)
    expected = 2 * E.reference_image("plane-d6") - E.reference_image("plane-d1")
    err, _ = E.error_image(img, expected)
    assert err < E.eps_for("plane-d6") * (E.DEFAULT_SPP / spp), err


def _multilight_floor(sc):
    d = sc.desc
    floor = [i for i in range(d.num_entities)
             if d.materials[d.entities[i].material].kd[0] == pytest.approx(0.885809)]
    assert len(floor) == 1
    return floor[0], np.array(d.materials[d.entities[floor[0]].material].kd[:])


@pytest.mark.parametrize("stem,selector", [("multilight-simple", 1), ("multilight-hierarchy", 2)])
def test_oracle_multilight_light_selectors(stem, selector):
    """CPU twin of the selector scenes: the oracle's flux-CDF ("simple") and
    light-hierarchy selectors (its own restatement of CDF.cpp, PointBvh.inl,
    LightHierarchy.cpp and light/light_selector.art, light_hierarchy.art)
    against the reference image, with the back-side environment term of the
    multilight scenes (see the module docstring), eps scaled by 1024/128."""
    from oracle import oracle_py as O

    spp = 128
    sc = load(stem)
    assert sc.desc.technique.light_selector == selector
    floor, kd = _multilight_floor(sc)
    cov = pixel_coverage(O.OracleScene(sc), sc, floor, grid=4)
    img, bad = render_oracle(sc, spp)
    expected = E.reference_image(stem) + 0.2 * kd[None, None, :] * cov[..., None]
    err, _ = E.error_image(img, expected.astype(np.float32))
    assert bad == 0
    assert err < E.eps_for(stem) * (E.DEFAULT_SPP / spp), err


CYCLES_BOX_MODEL = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "cycles_box_model.json")


def cycles_box_check(img, eps_scale=1.0):
    """The MODEL DIFFERENCE check of cycles-box (module docstring): background
    (environment-only) pixels at RunEvaluations' eps; the principled cube's
    mean over the reference image's equals the ratio derived from the two
    diffuse models (tests/golden/cycles_box_model.py: 0.9558) within 0.5 %;
    the image within 2 x eps."""
    with open(CYCLES_BOX_MODEL) as f:
        expected = json.load(f)["expected_ratio"]
    ref = E.reference_image("cycles-box")
    eps = E.eps_for("cycles-box") * eps_scale
    cube = ref.mean(axis=2) > 0.06  # everything brighter than the 0.0509 environment
    assert 0.2 < cube.mean() < 0.5
    bg_err, _ = E.error_image(img[~cube], ref[~cube])
    assert bg_err < eps, bg_err
    ratio = img[cube].mean() / ref[cube].mean()
    assert abs(ratio / expected - 1) < 5e-3, (ratio, expected)
    err, _ = E.error_image(img, ref)
    assert err < 2 * eps, err
    return err, ratio


def test_cycles_box_model_derivation():
    """The derived ratio (tests/golden/cycles_box_model.json) recomputes: the
    cube integrated numerically under the reference's principled diffuse lobe
    and under Cycles' (Blender 3.x: Disney 2015's split on the roughness input,
    algebraically Burley 2012's F_D90 form), at a coarser pixel grid and
    quadrature.  The Cycles-model cube matches Cycles' own image to 0.5 %
    (0.04 % measured), so the model difference is the diffuse lobe alone."""
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
    import cycles_box_model as M

    with open(CYCLES_BOX_MODEL) as f:
        committed = json.load(f)
    imgs = M.model_images(grid=2, models=(0, 1), quad=(48, 96))
    ref = E.reference_image("cycles-box")
    cube = ref.mean(axis=2) > 0.06
    ratio = imgs[0][cube].mean() / imgs[1][cube].mean()
    assert abs(ratio / committed["expected_ratio"] - 1) < 1e-3, (ratio, committed["expected_ratio"])
    assert abs(imgs[1][cube].mean() / ref[cube].mean() - 1) < 5e-3
    assert 0.94 < committed["expected_ratio"] < 0.97


def test_oracle_cycles_box_principled():
    """CPU twin of the cycles-box check at 128 spp (eps scaled by 1024/128)."""
    spp = 128
    sc = load("cycles-box")
    assert sc.desc.num_materials == 1 and sc.desc.materials[0].bsdf_type == 4  # principled
    img, bad = render_oracle(sc, spp)
    assert bad == 0
    cycles_box_check(img, E.DEFAULT_SPP / spp)


def test_externals_replace_by_name():
    """Parser.cpp:450-459 + Scene::addFrom: the including file's objects replace
    the external's objects of the same name (two-planes-mirror swaps the 'Back'
    BSDF of two-planes-base.json for a mirror)."""
    base_scene, mirror_scene = load("two-planes-plastic"), load("two-planes-mirror")
    base, mirror = base_scene.desc, mirror_scene.desc
    kinds = lambda d: sorted(d.materials[i].bsdf_type for i in range(d.num_materials))
    assert kinds(base) != kinds(mirror)
    assert base.num_entities == mirror.num_entities == 3


# ------------------------------------------------------------------ GPU tests
@pytest.fixture(scope="module")
def device():
    d = ignis_amd.Device(0)
    yield d
    d.close()


@pytest.mark.gpu
@pytest.mark.parametrize("stem", DIRECT)
def test_gpu_matches_reference_image(device, stem):
    """RunEvaluations.py's check as is: 1024 spp, err < predef_eps."""
    img, bad = render_device(device, load(stem), E.DEFAULT_SPP)
    err, _ = E.error_image(img, E.reference_image(stem))
    assert bad == 0
    assert err < E.eps_for(stem), err


@pytest.mark.gpu
def test_gpu_plane_d6_two_sided_lambert(device):
    img, _ = render_device(device, load("plane-d6"), E.DEFAULT_SPP)
    expected = 2 * E.reference_image("plane-d6") - E.reference_image("plane-d1")
    err, _ = E.error_image(img, expected)
    assert err < E.eps_for("plane-d6"), err
    # and the untransformed reference is clearly off (the effect is real)
    assert E.error_image(img, E.reference_image("plane-d6"))[0] > 100 * E.eps_for("plane-d6")


@pytest.mark.gpu
def test_gpu_cbox_d6_black_luminaire(device):
    with open(os.path.join(E.EVAL_DIR, "cbox-base.json")) as f:
        doc = json.load(f)
    doc["technique"] = {"type": "path", "max_depth": 6}
    assert doc["entities"][0]["name"] == "__entity_0" and doc["lights"][0]["entity"] == "__entity_0"
    doc["entities"][0]["bsdf"] = "__black"
    ref = E.reference_image("cbox-d6")
    img, _ = render_device(device, scene_from_doc(doc, E.EVAL_DIR), E.DEFAULT_SPP)
    err, _ = E.error_image(img, ref)
    assert err < E.eps_for("cbox-d6"), err
    # the scene as given: the luminaire lights itself through NEE (+16 %)
    full, _ = render_device(device, load("cbox-d6"), E.DEFAULT_SPP)
    assert full.mean() > 1.1 * ref.mean()


@pytest.mark.gpu
def test_gpu_flipped_prim_diffuse_mirror_symmetry(device):
    with open(os.path.join(E.EVAL_DIR, "flipped-prim-base.json")) as f:
        doc = json.load(f)
    doc["bsdfs"] = [{"type": "diffuse", "name": "base", "reflectance": [0.8, 0.8, 0.8]}]
    assert doc["entities"][0]["transform"] == [1, 0, 0, 0, 0, 1, 0, 0, 0, 0, -1, 0]
    doc["entities"][0]["transform"] = [1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0]
    img, _ = render_device(device, scene_from_doc(doc, E.EVAL_DIR), E.DEFAULT_SPP)
    expected = E.reference_image("flipped-prim-diffuse")[::-1]
    err, _ = E.error_image(img, expected)
    assert err < E.eps_for("flipped-prim-diffuse"), err


@pytest.mark.gpu
def test_gpu_cycles_box_principled(device):
    """Principled BSDF, point light by power and a constant environment given
    as colour expressions, against Blender Cycles' converged image at
    RunEvaluations' protocol (1024 spp): the MODEL DIFFERENCE check."""
    img, bad = render_device(device, load("cycles-box"), E.DEFAULT_SPP)
    assert bad == 0
    cycles_box_check(img)


@pytest.mark.gpu
@pytest.mark.parametrize("stem", MULTILIGHT)
def test_gpu_multilight_back_side_environment(device, stem):
    try:
        sc = load(stem)
    except ignis_amd.IgxError as e:
        pytest.skip(str(e))
    floor, kd = _multilight_floor(sc)
    device.upload(sc)
    cov = pixel_coverage(device, sc, floor)
    img, _ = render_device(device, sc, E.DEFAULT_SPP)
    expected = E.reference_image(stem) + 0.2 * kd[None, None, :] * cov[..., None]
    err, _ = E.error_image(img, expected.astype(np.float32))
    assert err < E.eps_for(stem), err


@pytest.mark.gpu
@pytest.mark.parametrize("stem", DIRECT + ["plane-d6", "cbox-d6", "flipped-prim-diffuse", "multilight",
                                           "multilight-simple", "multilight-hierarchy",
                                           "three-planes-glass", "three-planes-interface", "cycles-box"])
def test_gpu_matches_oracle_on_evaluation_scenes(device, stem):
    """Same scene, seed and spi on the HIP device and the oracle: per-path
    agreement up to float rounding, so the images agree far below the noise."""
    sc = load(stem)
    w, h = sc.film_size
    g, _ = render_device(device, sc, SPI)
    o, _ = render_oracle(sc, SPI)
    err, _ = E.error_image(g, o)
    assert err < 1e-3, err
    assert np.mean(np.abs(g - o) <= 1e-3 * np.abs(o) + 1e-5) >= 0.98
