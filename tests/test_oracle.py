"""Oracle vs. the reference's own known answers (CPU, no GPU needed)."""
import json
import math
import os

import numpy as np
import pytest

import ignis_amd
from oracle import oracle_py as O
from conftest import ENV_LIGHT, POINT_LIGHT, SPOT_LIGHT, flat_scene

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def load_golden(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


# ---- test_intersection.art KATs -------------------------------------------
@pytest.mark.parametrize("case", load_golden("intersection_kats.json")["triangles"], ids=lambda c: c["name"])
def test_triangle_kat(case):
    tri = np.array(case["v0"] + case["e1"] + case["e2"] + case["n"], np.float32)
    hit, tuv = O.intersect_tri(tri, case["ray"])
    assert hit == case["hit"]
    if hit:
        np.testing.assert_allclose(tuv, [case["t"], case["u"], case["v"]], atol=1e-6)


@pytest.mark.parametrize("case", load_golden("intersection_kats.json")["boxes"], ids=lambda c: c["name"])
def test_box_kat(case):
    hit, t = O.intersect_box(case["min"], case["max"], case["ray"])
    assert hit == case["hit"]
    if hit:
        assert t == pytest.approx(case["t"], abs=1e-6)


# ---- RNG: independent restatement of core/random.art in Python ------------
def _hash_combine(h, d):
    d &= 0xFFFFFFFF
    for s in (0, 8, 16, 24):
        h = ((h * 16777619) & 0xFFFFFFFF) ^ ((d >> s) & 0xFF)
    return h


def _seed(sample, it, frame, x, y, user):
    h = 0x811C9DC5
    for v in (sample, it, frame, x, y, user):
        h = _hash_combine(h, v)
    return h


def _tea(v0, v1):
    s = 0
    M = 0xFFFFFFFF
    for _ in range(4):
        s = (s + 0x9E3779B9) & M
        v0 = (v0 + ((((v1 << 4) & M) + 0xA341316C) ^ ((v1 + s) & M) ^ ((v1 >> 5) + 0xC8013EA4))) & M
        v1 = (v1 + ((((v0 << 4) & M) + 0xAD90777D) ^ ((v0 + s) & M) ^ ((v0 >> 5) + 0x7E95761E))) & M
    return v1


def _next_f32(seed, counter):
    x = _tea(seed, counter)
    bits = (x & 0x7FFFFF) | 0x3F800000
    return float(np.array([bits], np.uint32).view(np.float32)[0]) - 1.0


@pytest.mark.parametrize("args", [(0, 0, 0, 0, 0, 0), (3, 7, 1, 512, 333, 42), (7, 31, 0, 999, 999, -5)])
def test_rng_matches_python_restatement(args):
    import ctypes as C
    seed = O.lib().oracle_random_seed(*args)
    assert seed == _seed(*args)
    c = C.c_uint32(1)
    for k in range(1, 6):
        f = O.lib().oracle_next_f32(seed, C.byref(c))
        assert c.value == k + 1
        assert f == np.float32(_next_f32(seed, k))
        assert 0.0 <= f < 1.0


# ---- analytic integrator KATs (test_lights.py / test_init.py) ---------------
def _oracle_mean(scene_dict, size=200, spi=8):
    sc = ignis_amd.Scene.from_string(scene_dict)
    o = O.OracleScene(sc)
    fb, st = o.render(size, size, spi)
    img = fb.reshape(size, size, 3)
    pix = img.mean(axis=2)
    return float(pix.mean()), float(pix.std() / math.sqrt(pix.size)), st


ANALYTIC = load_golden("analytic_kats.json")["cases"]


@pytest.mark.parametrize("name,light", [("no_light", None), ("point", POINT_LIGHT), ("spot", SPOT_LIGHT), ("env", ENV_LIGHT)])
def test_oracle_analytic(name, light):
    mean, se, _ = _oracle_mean(flat_scene([light] if light else []))
    expected = ANALYTIC[name]["value"]
    assert abs(mean - expected) <= 5 * se + 1e-6, (mean, expected, se)


def test_oracle_empty_scene():
    sc = ignis_amd.Scene.from_string({})
    o = O.OracleScene(sc)
    fb, st = o.render(32, 24, 4)
    assert np.all(fb == 0)
    assert st["camera_rays"] == 32 * 24 * 4


def test_oracle_reproducible_and_spi_dependent():
    """test_reproducibility.py:5-20: same seed -> identical; different spi -> different."""
    sc = ignis_amd.Scene.from_string(flat_scene([POINT_LIGHT]))
    o = O.OracleScene(sc)
    a, _ = o.render(64, 64, 1, seed=42)
    b, _ = o.render(64, 64, 1, seed=42)
    np.testing.assert_array_equal(a, b)
    c, _ = o.render(64, 64, 4, seed=42)
    assert not np.allclose(a, c)


def test_oracle_thread_count_invariant(diamond_path):
    sc = ignis_amd.Scene.from_file(diamond_path)
    o = O.OracleScene(sc)
    a, _ = o.render(48, 48, 2, threads=1)
    b, _ = o.render(48, 48, 2, threads=5)
    np.testing.assert_array_equal(a, b)


def test_oracle_furnace_sphere():
    """White diffuse closed sphere in a constant environment: every pixel -> 1 (energy conservation)."""
    scene = {
        "technique": {"type": "path", "max_depth": 64},
        "camera": {"type": "perspective", "fov": 40, "near_clip": 0.1, "far_clip": 100,
                   "transform": [1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, -4, 0, 0, 0, 1]},
        "film": {"size": [64, 64]},
        "bsdfs": [{"type": "diffuse", "name": "white", "reflectance": [1, 1, 1]}],
        "shapes": [{"type": "sphere", "name": "S"}],
        "entities": [{"name": "S", "shape": "S", "bsdf": "white"}],
        "lights": [{"type": "env", "name": "E", "radiance": [1, 1, 1]}],
    }
    sc = ignis_amd.Scene.from_string(scene)
    o = O.OracleScene(sc)
    fb, _ = o.render(64, 64, 16)
    pix = fb.reshape(64, 64, 3).mean(axis=2)
    assert abs(pix.mean() - 1.0) < 0.02
