"""Workload for rocprofv3 counter passes: the bench's iterations of a scene
(default diamond 1000x1000, spi 8), batched by igx_render_iterations like the
bench, without timing or instrumentation, so every k_extend dispatch is the
same kernel with the same path count the bench times; one warm-up render of
the same shape first (tools/profile_summary.py drops its dispatches).
Usage: pmc_run.py [iterations] [scene file under scenes/] [device options as JSON] [square film size]
(the size overrides the scene's film as bench.py's suite does for the config-5 stand-in)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ignis-masterthesis_amd"))
import ignis_amd  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 2
scene = ignis_amd.Scene.from_file(os.path.join(ROOT, "scenes", sys.argv[2] if len(sys.argv) > 2 else "diamond_scene.json"))
W, H = scene.film_size
if len(sys.argv) > 4 and int(sys.argv[4]) > 0:
    W = H = int(sys.argv[4])
dev = ignis_amd.Device(0)
import json  # noqa: E402
for k, v in (json.loads(sys.argv[3]) if len(sys.argv) > 3 else {}).items():
    dev.set_option(k, v)
dev.upload(scene)
p = ignis_amd.RenderParams()
p.width, p.height, p.spi = W, H, 8
p.iteration = 0
# warm-up with the same shape (slot buffers allocated, tables touched), as the
# bench does before its timed call; tools/profile_summary.py keeps the second
# half of each kernel's dispatches (the measured render)
dev.render_iterations(p, iters)
dev.synchronize()
dev.reset_stats()
dev.render_iterations(p, iters)  # batched like the bench's frame
dev.synchronize()
st = dev.stats()
print({k: st[k] for k in ("camera_rays", "bounce_rays", "shadow_rays", "launches_extend", "extend_rays")}, flush=True)
dev.close()
