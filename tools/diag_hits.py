"""Dev tool: closest-hit parity of trace_hits against the oracle on the
diamond scene's camera and random rays (tests/test_gpu.py's rays) under a few
device options (IGX_DIAG_OPTS, a JSON list of option dicts; default one set
of defaults), printing the rays whose barycentrics disagree."""
import json, os, sys, numpy as np
sys.path.insert(0, "tests"); sys.path.insert(0, "ignis-masterthesis_amd"); sys.path.insert(0, ".")
import ignis_amd
from test_gpu import random_rays, camera_rays
import oracle.oracle_py as O
sc = ignis_amd.Scene.from_file("scenes/diamond_scene.json")
orc = O.OracleScene(sc)
sets = [(camera_rays(sc, 320, 320, jitter=0.37), 0x1), (random_rays(sc, 100000), 0x4)]
for opts in json.loads(os.environ.get("IGX_DIAG_OPTS", "[{}]")):
    d = ignis_amd.Device(0)
    for k, v in opts.items(): d.set_option(k, v)
    d.upload(sc)
    for rays, flags in sets:
        eo, to = orc.trace_hits(rays, flags)
        eg, tg = d.trace_hits(rays, flags)
        same = np.all(eg == eo, axis=1) & (eo[:, 0] >= 0)
        bad = np.flatnonzero(same & (np.abs(tg[:, 1:] - to[:, 1:]).max(1) > 1e-3))
        print(opts, flags, "bad", bad.tolist())
        for i in bad[:4]:
            print(" ray", rays[i].tolist(), "gpu", eg[i].tolist(), tg[i].tolist(), "orc", eo[i].tolist(), to[i].tolist())
    d.close()
