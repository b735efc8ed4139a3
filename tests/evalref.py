"""The reference's image-evaluation protocol (TEST INFRASTRUCTURE).

Restates `scripts/RunEvaluations.py` of the reference: the error metric
`error_image` (lines 80-87: RelSE where the reference pixel is non-zero, AbsSE
where it is zero, mean of the error clamped at its 99th percentile), the
per-scene tolerances `predef_eps` (lines 91-114, default 1e-3 at line 153), the
rendering protocol of `evaluate_target` (lines 41-55: `step()` until
SampleCount >= spp, image = framebuffer / IterationCount, non-finite pixels set
to 0 after being reported, lines 157-164) and the default of 1024 spp
(line 231).  The reference images are the reference's own
`scenes/evaluation/references/*.exr`, copied as data by
`tests/golden/make_eval_fixtures.py` into `scenes/evaluation/references/`.
"""
import json
import os

import numpy as np

from exr_read import read_rgb

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EVAL_DIR = os.path.join(ROOT, "scenes", "evaluation")
DEFAULT_EPS = 1e-3
DEFAULT_SPP = 1024

PREDEF_EPS = {
    "cbox-d1": 5e-3, "cbox-d6": 5e-3, "cycles-lights": 5e-2, "cycles-principled": 5e-2,
    "cycles-tex": 1e-2, "cycles-sun": 1e-2, "room": 1e-3, "volume": 5e-3, "env4k": 8e-2,
    "env4k-nocdf": 8e-2, "env4k-nomisc": 8e-2, "multilight-uniform": 3e-4,
    "multilight-simple": 3e-4, "multilight-hierarchy": 3e-4, "plane-array-klems-front": 2e-2,
    "plane-array-klems-back": 2e-2, "plane-array-tensortree-front": 2e-2,
    "plane-array-tensortree-back": 2e-2, "sphere-light-ico": 2e-3, "sphere-light-ico-nopt": 2e-3,
    "sphere-light-uv": 2e-3, "sphere-light-pure": 3e-3,
}


def error_image(img, ref):
    """RunEvaluations.py:80-87 -> (mean clamped error, normalised error image)."""
    mask = ref != 0
    err = np.zeros_like(ref)
    err[mask] = np.square((img[mask] - ref[mask]) / ref[mask])
    err[~mask] = np.square(img[~mask])
    mx = np.percentile(err, 99)
    avg = float(np.average(np.clip(err, 0, mx)))
    return avg, (np.clip(err / mx, 0, 1) if mx != 0 else np.zeros_like(ref))


def eps_for(stem):
    return PREDEF_EPS.get(stem, DEFAULT_EPS)


def reference_path(stem):
    with open(os.path.join(EVAL_DIR, "references.json")) as f:
        return os.path.join(ROOT, "scenes", json.load(f)[stem])


def reference_image(stem):
    return read_rgb(reference_path(stem)).astype(np.float32)


def scene_path(stem):
    return os.path.join(EVAL_DIR, stem + ".json")


def sanitize(img):
    """Non-finite pixels count as errors in RunEvaluations (reported, then zeroed)."""
    img = np.array(img, dtype=np.float32, copy=True)
    bad = ~np.isfinite(img)
    img[bad] = 0
    return img, int(bad.sum())
