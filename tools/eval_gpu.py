"""Render the reference's evaluation scenes on the HIP device and score them with
RunEvaluations' metric (tests/evalref.py).  Diagnostic tool for the GPU box:

    python tools/eval_gpu.py [spp] [scene ...]

Writes gpurun_out/eval_<spp>.npz (images) and prints one line per scene.
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ignis-masterthesis_amd"), ROOT, os.path.join(ROOT, "tests")]

import ignis_amd  # noqa: E402
import evalref as E  # noqa: E402


def main():
    spp = int(sys.argv[1]) if len(sys.argv) > 1 else E.DEFAULT_SPP
    with open(os.path.join(E.EVAL_DIR, "references.json")) as f:
        stems = sorted(json.load(f))
    if len(sys.argv) > 2:
        stems = sys.argv[2:]
    dev = ignis_amd.Device(0)
    out = {}
    for stem in stems:
        try:
            sc = ignis_amd.Scene.from_file(E.scene_path(stem))
            dev.upload(sc)
        except Exception as e:  # unsupported scene feature
            print(f"{stem:28s} LOAD {e}", flush=True)
            continue
        w, h = sc.film_size
        spi = 8
        t = time.time()
        dev.clear()
        p = ignis_amd.RenderParams()
        p.width, p.height, p.spi = w, h, spi
        dev.render_iterations(p, (spp + spi - 1) // spi)
        fb, it = dev.framebuffer(w * h * 3)
        img, bad = E.sanitize(fb.reshape(h, w, 3) / it)
        dt = time.time() - t
        ref = E.reference_image(stem)
        err, _ = E.error_image(img, ref)
        eps = E.eps_for(stem)
        out[stem] = img
        print(f"{stem:28s} err {err:.3e} eps {eps:.0e} {'PASS' if err < eps else 'FAIL'} x{err / eps:6.2f} "
              f"mean {img.mean():.4f} ref {ref.mean():.4f} nonfinite {bad} {dt:.2f}s", flush=True)
    dev.close()
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    np.savez_compressed(os.path.join(ROOT, "gpurun_out", f"eval_{spp}.npz"), **out)


if __name__ == "__main__":
    main()
