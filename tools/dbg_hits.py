import os, sys
sys.path.insert(0, "ignis-masterthesis_amd"); sys.path.insert(0, "."); sys.path.insert(0, "tests")
import numpy as np, ignis_amd
from oracle import oracle_py as O
import test_gpu as T
sc = ignis_amd.Scene.from_file("scenes/primitives.json")
dev = ignis_amd.Device(0); dev.upload(sc); orc = O.OracleScene(sc)
rays = T.random_rays(sc, 50000, 7)
(eg, tg), (eo, to) = dev.trace_hits(rays, 4), orc.trace_hits(rays, 4)
same = np.all(eg == eo, axis=1) & (eo[:, 0] >= 0)
bad = np.flatnonzero(same & (np.abs(tg[:, 1:] - to[:, 1:]).max(axis=1) > 1e-3))
print("n bad", len(bad), bad)
for i in bad[:4]:
    e1, t1 = dev.trace_hits(rays[i:i + 1], 4)
    blk = (i // 256) * 256
    e2, t2 = dev.trace_hits(rays[blk:blk + 256], 4)
    e3, t3 = dev.trace_hits(rays[i - (i % 64): i - (i % 64) + 64], 4)
    print(i, "full", eg[i], tg[i], "single", e1[0], t1[0], "block", e2[i - blk], t2[i - blk], "wave", e3[i % 64], t3[i % 64], "oracle", to[i])
    # which other ray in the wave has this u,v?
    w0 = i - (i % 64)
    print("   wave lanes with same u:", [j for j in range(w0, w0 + 64) if abs(to[j, 1] - tg[i, 1]) < 1e-6])
