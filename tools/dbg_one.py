import sys
sys.path.insert(0, "ignis-masterthesis_amd"); sys.path.insert(0, "."); sys.path.insert(0, "tests")
import numpy as np, ignis_amd
import test_gpu as T
sc = ignis_amd.Scene.from_file("scenes/primitives.json")
dev = ignis_amd.Device(0); dev.upload(sc)
rays = T.random_rays(sc, 50000, 7)
i = int(sys.argv[1]) if len(sys.argv) > 1 else 11447
e, t = dev.trace_hits(rays, 4)
print(e[i], t[i], flush=True)
