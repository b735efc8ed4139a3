#!/usr/bin/env python3
"""Benchmark of the wavefront traversal-and-shade loop on MI355X.

Metric (BASELINE.json): Mrays/s (primary + secondary) at fixed spp, per-pixel
L2 vs the CPU reference.  Workload = BASELINE config 2: scenes/diamond_scene.json,
1000x1000 film, 256 spp as 32 iterations of spi 8, path tracer max_depth 64,
seed 0.  One "step" = one full 256-spp frame.  Rays = camera rays + bounce rays
(closest-hit traversals) + valid shadow rays (any-hit traversals), counted on
the device.

Multi-GPU (torchrun, one rank per GPU): the film is cut into square tiles
(40 px for 1000-px films: a tile column count coprime with N, shard.balanced_tile)
dealt round-robin to the ranks (tile t -> rank t % N); every rank renders all 32
iterations of its tiles, packs them, and an RCCL gather over xGMI brings the
packed tiles to rank 0, which assembles the frame.  Total work is fixed, so
scaling is "strong".  At every N the line also carries `config5`: BASELINE
config 5's stand-in (S-deep at 4096x4096, 64 spp) rendered the
same way, tile-sharded over the N ranks and gathered; at N > 1 both carry a
per-rank breakdown (`ranks`: frame / pack / gather ms and rays per rank) and
`frame_equals_single_gpu` (the gathered frame against rank 0's whole-frame
render, bit for bit).

Output: ONE JSON line on rank 0.
"""
import argparse
import ctypes as C
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "ignis-masterthesis_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--scene", default=os.path.join(ROOT, "scenes", "diamond_scene.json"))
    ap.add_argument("--spp", type=int, default=256)
    ap.add_argument("--spi", type=int, default=8)
    ap.add_argument("--size", type=int, default=0, help="square film size overriding the scene's (config 5: 4096)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU baseline sample length")
    ap.add_argument("--suite", type=int, default=1, help="also measure the other §8d scenes (N=1 only)")
    ap.add_argument("--check-frame", action="store_true", help="(default at N > 1; kept for older scripts)")
    ap.add_argument("--no-check-frame", action="store_true",
                    help="N>1: skip rank 0's whole-frame render that checks the gathered frame bit for bit")
    ap.add_argument("--config5", type=int, default=1,
                    help="also measure BASELINE config 5's stand-in (S-deep 4096x4096, 64 spp) tile-sharded over the N ranks")
    ap.add_argument("--config5-steps", type=int, default=2, help="timed frames of the config-5 line")
    ap.add_argument("--isolated", type=int, default=1,
                    help="after the timed frames, one more frame with concurrent_chunks 0 for the dominant kernel's own "
                         "launch duration (roofline.isolated); 0 for rocprofv3 runs whose average should be the timed frames'")
    return ap.parse_args()


# Tables up to half the 256 MiB Infinity Cache count as on-chip: a table stays resident only while it and
# everything streamed between two uses of a line fit the cache (MI355X_MICROARCH.md, Infinity Cache)
MALL_BYTES = 128 << 20
# N > 1: a rank holds two handles, each with ONE stream slot (option
# stream_slots) sized to the rank's share of a frame when that is one chunk
# (the diamond: N = 2: 128 M paths = 37 GB per handle, 8: 9.3 GB), two
# otherwise (rank_stream_slots).  A budget below the share
# splits a frame into chunks and costs time (slot_budget_mb 20000 at N = 2:
# 67.3 vs 55.2 ms per rank frame, profiles/r03_exp_classes_regroup_slots.log);
# IGX_SLOT_BUDGET_MB caps it anyway (0 = auto)
SLOT_BUDGET_MB = int(os.environ.get("IGX_SLOT_BUDGET_MB", "0"))
# the rehearsal puts every rank on GPU 0: each rank's two handles then get an
# equal share of half the device memory for their stream slots
def rehearsal_slot_budget_mb(torch, n):
    return max(256, int(torch.cuda.get_device_properties(0).total_memory * 0.5 / (2 * n) / 2**20))


# paths of one chunk (igx_device.hip MAX_CHUNK_PATHS)
MAX_CHUNK_PATHS = 1 << 27


def rank_stream_slots(W, H, tile, n, spi, iters):
    """Stream slots per device handle of a rank at N > 1: 1 when the rank's
    share of a frame (its tiles, all iterations) fits one chunk, else 2.  With
    one slot per handle the chunks of a multi-chunk share run back to back and
    each chunk's tail is exposed: S-deep 4096^2, 8 iterations, N = 2: a rank
    frame of 391.5 ms against 309.1 ms for the same path count as a 2896^2
    film with two slots (profiles/r04_probe_chunks_tiles.log)."""
    from ignis_amd import shard
    share = shard.max_tiles_per_rank(W, H, tile, n) * tile * tile * spi * iters
    return 1 if share <= MAX_CHUNK_PATHS else 2


def algorithmic_bytes(inst, st):
    """Algorithmic HBM bytes of the dominant kernel's launches.

    Streams, on every scene:
    * fused k_extend: per closest-hit ray 52 B path state read (camera rays:
      none, bounce 0 builds them, fuse_generate) and its 16 B radiance slot
      read + written (camera rays: written only); 52 B per surviving path and
      48 B per shadow ray written;
    * split k_trace: 32 B ray read + 20 B hit record written per ray.
    Scene tables: when the traversal + shading tables fit the 256 MiB
    Infinity Cache (diamond, primitives, S-deep, S-soup-1M) they are fetched
    from HBM about once and every further node / triangle / vertex read is an
    on-chip hit (LDS on the LDS-staged diamond), so they add nothing per ray.
    Beyond it (S-soup-16M, 1.8 GB) every visit is a potential HBM read:
    node_bytes per node + 64 B per instance + 48 B per triangle per ray, plus
    (fused) 288 B of shading fetches per hit.
    Returns (total bytes, per-ray bytes, memory-system bytes): the last counts
    every table read the kernel issues whatever level serves it (the
    round-1 'algorithmic' figure, a work rate, not an HBM figure)."""
    n = max(inst["_rays_ext"], 1)
    bvh = float(st.get("node_bytes", 64)) * inst["node_visits"] / n + 64.0 * inst["leaf_visits"] / n + 48.0 * inst["tri_tests"] / n
    shade = 288.0 * inst["_hits"] / n
    resident = st["table_bytes"] + st["shading_bytes"] <= MALL_BYTES
    if st["launches_trace"] > 0:
        stream = 32 + 20
        per_ray = stream + (0 if resident else bvh)
        return st["extend_rays"] * per_ray, per_ray, st["extend_rays"] * (stream + bvh)
    shadow_wf = st["shadow_rays"] - st["tail_shadow_rays"]
    cam = st["camera_rays"]
    streams = (st["extend_rays"] - cam) * (52 + 32) + cam * 16 + st["extend_paths_out"] * 52 + shadow_wf * 48
    tables = st["extend_rays"] * (bvh + shade)
    total = streams + (0 if resident else tables)
    return total, total / max(st["extend_rays"], 1), streams + tables


def load_pmc(n_gpus, scene="diamond_scene", kernel="extend"):
    """Per-launch HBM traffic of the dominant kernel (k_extend, or k_trace on
    split scenes) from the committed rocprofv3 PMC summary of the same workload
    (profiles/pmc_<kernel>[_<scene>].json, tools/profile_summary.py)."""
    name = f"pmc_{kernel}.json" if scene == "diamond_scene" else f"pmc_{kernel}_{scene}.json"
    path = os.path.join(ROOT, "profiles", name)
    if n_gpus != 1 or not os.path.exists(path):
        return None
    try:
        with open(path) as f:
            return json.load(f)
    except Exception:
        return None


def load_rocprof(scene_key, split, kernel=None):
    """Average duration (us) of the dominant kernel in the newest committed
    rocprofv3 --kernel-trace --stats summary of the same workload:
    profiles/rNN_kernel_stats.csv (headline diamond) or
    profiles/rNN_<key>_kernel_stats.csv (suite lines, tools/gpu_profile_suite.sh)."""
    import csv
    import re
    pat = re.compile(r"^r(\d\d)_kernel_stats\.csv$" if scene_key == "diamond_scene" else
                     r"^r(\d\d)_" + re.escape(scene_key) + r"_kernel_stats\.csv$")
    d = os.path.join(ROOT, "profiles")
    files = sorted((f for f in os.listdir(d) if pat.match(f)), key=lambda f: int(pat.match(f).group(1)))
    if not files:
        return None
    want = kernel or ("k_trace_refill<" if split else "k_extend<")
    with open(os.path.join(d, files[-1])) as f:
        for r in csv.DictReader(f):
            if want in r["Name"]:
                return {"file": "profiles/" + files[-1], "avg_us": round(float(r["AverageNs"]) / 1e3, 2),
                        "calls": int(r["Calls"])}
    return None


SQ_PROFILES = {"diamond_scene": "r06_sq_diamond.json", "s_deep": "r06_sq_sdeep.json", "s_soup_16m": "r06_sq_soup16.json"}


def sq_limiter(scene_key, kernel):
    """Where the kernel's wave cycles go, from the committed round-6 SQ/TCC
    counter summary of the same workload (tools/gpu_pmc_sq.sh ->
    tools/pmc_sq_summary.py): SQ_WAIT_ANY (waiting on a memory or LDS counter),
    SQ_WAIT_INST_ANY (waiting to issue) and SQ_ACTIVE_INST_ANY (issuing) over
    SQ_WAVE_CYCLES, VALU lane use SQ_THREAD_CYCLES_VALU / (64 SQ_ACTIVE_INST_VALU)
    and the L2 hit rate TCC_HIT / (TCC_HIT + TCC_MISS)."""
    name = SQ_PROFILES.get(scene_key)
    path = os.path.join(ROOT, "profiles", name) if name else None
    if not path or not os.path.exists(path):
        return "no SQ counter profile committed for this workload"
    with open(path) as f:
        ks = json.load(f)["kernels"]
    for k, v in ks.items():
        if k.split("<")[0] == kernel:
            return (f"wave cycles {v['wait_any']:.0%} waiting on memory/LDS, {v['wait_inst_any']:.0%} waiting to issue, "
                    f"{v['active_inst_any']:.0%} issuing; VALU lane use {v['lane_util']:.0%}; L2 hit {v['l2_hit']:.0%} "
                    f"(profiles/{name})")
    return f"{kernel} not in profiles/{name}"


def roofline(dev, st, render_one, n_gpus, scene_key):
    """Roofline object of the dominant kernel: algorithmic HBM bytes (visit
    counts from an instrumented, untimed pass) over its HIP-event launch time,
    next to the PMC-measured HBM traffic of the same kernel."""
    dev.reset_stats()
    dev.set_option("instrument", 1)
    dev.clear()
    render_one()
    inst = dev.stats()
    dev.set_option("instrument", 0)
    inst["_rays_ext"] = inst["camera_rays"] + inst["bounce_rays"]
    inst["_hits"] = inst["shaded_hits"]
    alg_bytes, bytes_per_ray, mem_bytes = algorithmic_bytes(inst, st)
    split = st["launches_trace"] > 0
    launches = max(st["launches_trace"] if split else st["launches_extend"], 1)
    avg_launch_s = (st["ms_trace"] if split else st["ms_extend"]) / 1e3 / launches
    achieved = (alg_bytes / launches) / avg_launch_s / 1e9 if avg_launch_s > 0 else 0.0
    pmc = load_pmc(n_gpus, scene_key, "trace" if split else "extend")
    traffic = float(pmc["hbm_bytes_per_launch"]) if pmc else None
    simd = inst["node_visits"] / max(1, 64 * inst["wave_node_iters"])
    resident = st["table_bytes"] + st["shading_bytes"] <= MALL_BYTES
    out = {
        "bound": "hbm",
        "kernel": "k_trace (closest-hit traversal)" if split else "k_extend (closest-hit traversal + shading, fused)",
        "achieved": round(achieved, 1),
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBS, 4),
        "traffic": traffic,
        # measured HBM bandwidth of the same launches (PMC bytes / HIP-event time)
        "traffic_gbs": round(traffic / avg_launch_s / 1e9, 1) if traffic and avg_launch_s > 0 else None,
        "frac_traffic": round(traffic / avg_launch_s / 1e9 / HBM_PEAK_GBS, 4) if traffic and avg_launch_s > 0 else None,
        "traffic_raw": {k: pmc[k] for k in ("fetch_size_kib_per_launch", "write_size_kib_per_launch")} if pmc else None,
        "algorithmic_bytes_per_launch": round(alg_bytes / launches, 1),
        # > 1: bytes the counters see beyond the algorithmic count (table fetches
        # that miss L2, counted as on chip when the tables fit the Infinity Cache)
        "traffic_over_algorithmic": round(traffic / (alg_bytes / launches), 2) if traffic and alg_bytes > 0 else None,
        "bytes_per_ray": round(bytes_per_ray, 1),
        "tables_on_chip": bool(resident),
        "table_bytes": int(st["table_bytes"] + st["shading_bytes"]),
        # every table read the kernel issues, whatever serves it (LDS, L2, Infinity Cache, HBM)
        "memory_system_gbs": round((mem_bytes / launches) / avg_launch_s / 1e9, 1) if avg_launch_s > 0 else None,
        "visits_per_ray": {"nodes": round(inst["node_visits"] / max(1, inst["_rays_ext"]), 2),
                           "instances": round(inst["leaf_visits"] / max(1, inst["_rays_ext"]), 2),
                           "triangles": round(inst["tri_tests"] / max(1, inst["_rays_ext"]), 2)},
        "simd_efficiency": round(simd, 3),
        "avg_launch_us": round(avg_launch_s * 1e6, 2),
        "launches": launches,
    }
    # split schedule: the committed profile is of the trace kernel alone
    # (overlap_shadow 0), compared with roofline["isolated"] (suite_line)
    rp = load_rocprof(scene_key, split) if n_gpus == 1 and not split else None
    if rp:
        # the same quantities over the committed rocprof average of the same kernel and workload
        t = rp["avg_us"] * 1e-6
        out["rocprof"] = dict(rp, frac=round(alg_bytes / launches / t / 1e9 / HBM_PEAK_GBS, 4),
                              frac_traffic=round(traffic / t / 1e9 / HBM_PEAK_GBS, 4) if traffic else None)
    out["_inst"] = inst  # visit counts for shadow_roofline (dropped before the line is printed)
    sq = sq_limiter(scene_key, "k_trace_refill" if split else "k_extend")
    out["limiter"] = (f"not HBM: tables on chip, divergent per-lane traversal, node loop at {simd:.0%} SIMD efficiency; {sq}"
                      if resident else f"dependent node-fetch latency: node loop at {simd:.0%} SIMD efficiency; {sq}")
    return out


def isolated_extend(dev, render_frame, roof):
    """Fused schedule with concurrent chunks: the timed frames run two chunks'
    bounces at once (igx_device.hip render_chunks_concurrent), so a k_extend
    launch's HIP-event duration includes time shared with the other chunk's
    kernels.  One more frame with concurrent_chunks 0 (untimed for `value`)
    gives the kernel's own launch duration, reported next to the timed one."""
    dev.reset_stats()
    dev.set_option("timing", 1)
    dev.set_option("concurrent_chunks", 0)
    render_frame()
    dev.synchronize()
    si = dev.stats()
    dev.set_option("concurrent_chunks", 1)
    dev.set_option("timing", 0)
    t_iso = si["ms_extend"] / 1e3 / max(1, si["launches_extend"])
    roof["_si"] = si  # the same run's k_shadow launches (fused_shadow_roofline; dropped before printing)
    per_launch = roof["algorithmic_bytes_per_launch"]
    roof["isolated"] = {"avg_launch_us": round(t_iso * 1e6, 2),
                        "frac": round(per_launch / t_iso / 1e9 / HBM_PEAK_GBS, 4) if t_iso > 0 else None,
                        "frac_traffic": round(roof["traffic"] / t_iso / 1e9 / HBM_PEAK_GBS, 4) if t_iso > 0 and roof["traffic"] else None,
                        "note": "k_extend with concurrent_chunks 0 (each chunk's bounces alone on the chip): the kernel's own "
                                "launch duration; the timed frames overlap one chunk's last bounces with the next chunk's first"}


def shadow_roofline(st, inst, si, scene_key):
    """Roofline object of the split schedule's any-hit kernel (k_shadow_refill):
    per shadow ray 32 B of ray read, at most 48 B more for an unoccluded one
    (its colour, and the radiance slot read and written), plus -- tables beyond
    the Infinity Cache -- node_bytes per node, 64 B per instance and 48 B per
    triangle the any-hit walk visits (instrumented pass); over the kernel's own
    launch time (the overlap_shadow 0 run `si`), next to the PMC traffic of the
    committed profile of the same workload."""
    ns = max(1, inst["shadow_rays"])
    resident = st["table_bytes"] + st["shading_bytes"] <= MALL_BYTES
    tables = (float(st.get("node_bytes", 64)) * inst["shadow_node_visits"] + 64.0 * inst["shadow_leaf_visits"] +
              48.0 * inst["shadow_tri_tests"]) / ns
    per_ray = 32 + 48 + (0 if resident else tables)
    launches = max(1, si["launches_shadow"])
    t = si["ms_shadow"] / 1e3 / launches
    per_launch = si["shadow_rays"] * per_ray / launches
    pmc = load_pmc(1, scene_key, "shadow_refill")
    traffic = float(pmc["hbm_bytes_per_launch"]) if pmc else None
    out = {"bound": "hbm", "kernel": "k_shadow_refill (any-hit traversal, persistent lanes)",
           "achieved": round(per_launch / t / 1e9, 1) if t > 0 else None, "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": round(per_launch / t / 1e9 / HBM_PEAK_GBS, 4) if t > 0 else None, "traffic": traffic,
           "frac_traffic": round(traffic / t / 1e9 / HBM_PEAK_GBS, 4) if traffic and t > 0 else None,
           "algorithmic_bytes_per_launch": round(per_launch, 1), "bytes_per_ray": round(per_ray, 1),
           "traffic_over_algorithmic": round(traffic / per_launch, 2) if traffic and per_launch > 0 else None,
           "visits_per_ray": {"nodes": round(inst["shadow_node_visits"] / ns, 2),
                              "instances": round(inst["shadow_leaf_visits"] / ns, 2),
                              "triangles": round(inst["shadow_tri_tests"] / ns, 2)},
           "avg_launch_us": round(t * 1e6, 2), "launches": launches,
           "limiter": "dependent node-fetch latency of the any-hit walk; " + sq_limiter(scene_key, "k_shadow_refill"),
           "note": "the kernel's own launches (overlap_shadow 0); 48 B per ray counted as if every shadow ray were unoccluded"}
    rp = load_rocprof(scene_key, True, "k_shadow_refill<")
    if rp:
        tr = rp["avg_us"] * 1e-6
        out["rocprof"] = dict(rp, frac=round(per_launch / tr / 1e9 / HBM_PEAK_GBS, 4),
                              frac_traffic=round(traffic / tr / 1e9 / HBM_PEAK_GBS, 4) if traffic else None)
    return out


def fused_shadow_roofline(st, inst, si, scene_key):
    """Roofline object of the fused schedule's any-hit kernel (k_shadow): per
    shadow ray the 32 B ray read, and for an unoccluded one its 16 B colour plus
    the 16 B radiance slot read and written (tables: LDS-staged or on chip, no
    per-ray HBM bytes on the scenes that run fused), over the kernel's own
    launch time (the concurrent_chunks 0 run `si` of isolated_extend), next to
    the PMC traffic of the committed profile (profiles/pmc_shadow.json).  The
    per-class split (stream class A: rays that cross no enclosing entity's box,
    B: the rest, shadow_class_b) comes from the instrumented pass."""
    rays = max(1, si["shadow_rays"] - si["tail_shadow_rays"])
    launches = max(1, si["launches_shadow"])
    t = si["ms_shadow"] / 1e3 / launches
    g, it, vi, cy, oc, nr = (list(inst["shadow_class_" + k]) for k in ("groups", "node_iters", "node_visits", "cycles", "occluded", "rays"))
    occl = sum(oc) / max(1, sum(nr))  # occluded share of the k_shadow rays (instrumented pass; partial groups' padding lanes excluded)
    per_ray = 32 + 48 * (1 - occl)
    per_launch = rays * per_ray / launches
    pmc = load_pmc(1, scene_key, "shadow")
    traffic = float(pmc["hbm_bytes_per_launch"]) if pmc else None
    classes = {}
    for k, name in enumerate(("A", "B")):
        if g[k] == 0:
            continue
        classes[name] = {"groups": g[k], "cycle_share": round(cy[k] / max(1, sum(cy)), 3),
                         "wave_node_iters_per_group": round(it[k] / g[k], 2),
                         "simd_efficiency": round(vi[k] / max(1, 64 * it[k]), 3),
                         "rays": nr[k], "occluded_share": round(oc[k] / max(1, nr[k]), 3)}
    out = {"bound": "hbm", "kernel": "k_shadow (any-hit traversal of the fused schedule's shadow rays)",
           "achieved": round(per_launch / t / 1e9, 1) if t > 0 else None, "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": round(per_launch / t / 1e9 / HBM_PEAK_GBS, 4) if t > 0 else None, "traffic": traffic,
           "frac_traffic": round(traffic / t / 1e9 / HBM_PEAK_GBS, 4) if traffic and t > 0 else None,
           "algorithmic_bytes_per_launch": round(per_launch, 1), "bytes_per_ray": round(per_ray, 1),
           "traffic_over_algorithmic": round(traffic / per_launch, 2) if traffic and per_launch > 0 else None,
           "visits_per_ray": {"nodes": round(inst["shadow_node_visits"] / max(1, inst["shadow_rays"]), 2),
                              "triangles": round(inst["shadow_tri_tests"] / max(1, inst["shadow_rays"]), 2)},
           "avg_launch_us": round(t * 1e6, 2), "launches": launches, "ms_per_frame": round(si["ms_shadow"], 3),
           # the timed frames' launches (each shares the chip with the other chunk's k_extend):
           # what the rocprof average below is over
           "avg_launch_us_timed": round(st["ms_shadow"] * 1e3 / max(1, st["launches_shadow"]), 2),
           "classes": classes,
           "limiter": "the divergent any-hit walk below the HBM roof it is priced against (tables LDS-staged; "
                      "class B's node loop, see classes); " + sq_limiter(scene_key, "k_shadow"),
           "note": "the kernel's own launches (concurrent_chunks 0); classes: per shadow stream class, instrumented pass"}
    rp = load_rocprof(scene_key, False, "k_shadow<")
    if rp:
        tr = rp["avg_us"] * 1e-6
        out["rocprof"] = dict(rp, frac=round(per_launch / tr / 1e9 / HBM_PEAK_GBS, 4),
                              frac_traffic=round(traffic / tr / 1e9 / HBM_PEAK_GBS, 4) if traffic else None)
    return out


def suite_line(ignis_amd, dev_index, path, spi, iters, size=None, isolated=True):
    """Short single-GPU measurement of another scene of SURVEY.md §8d (load and
    BVH build excluded): Mrays/s over `iters` iterations after one warm-up,
    plus the dominant kernel's roofline on that scene.  `size` overrides the
    scene's film (the camera keeps its horizontal field of view)."""
    t_load = time.perf_counter()
    scene = ignis_amd.Scene.from_file(path)
    W, H = size or scene.film_size
    dev = ignis_amd.Device(dev_index)
    dev.upload(scene)
    t_load = time.perf_counter() - t_load
    p = ignis_amd.RenderParams()
    p.width, p.height, p.spi = W, H, spi
    dev.render_iterations(p, iters)  # warm-up with the timed call's shape (slot buffers sized)
    dev.synchronize()
    dev.reset_stats()
    dev.set_option("timing", 1)
    t0 = time.perf_counter()
    p.iteration = 1
    dev.render_iterations(p, iters)
    dev.synchronize()
    dt = time.perf_counter() - t0
    p.iteration = 0
    st = dev.stats()
    dev.set_option("timing", 0)
    rays = st["camera_rays"] + st["bounce_rays"] + st["shadow_rays"]
    # profiles/ key of the suite line: scene stem, plus the film size when overridden (config 5: s_deep_4096)
    key = os.path.splitext(os.path.basename(path))[0] + (f"_{size[0]}" if size else "")
    line = {"scene": os.path.basename(path), "width": W, "height": H, "spi": spi, "iterations": iters,
            "value": round(rays / dt / 1e6, 2), "unit": "Mrays/s", "ms_per_iteration": round(dt / iters * 1e3, 3),
            "load_and_build_s": round(t_load, 2), "bvh_depth": st["bvh_depth"],
            "roofline": roofline(dev, st, lambda: dev.render(p), 1, key)}
    if st["launches_trace"] > 0:
        # split schedule: k_trace_refill shares the chip with the shadow rays of the
        # previous bounce (option overlap_shadow), so its launch durations include
        # shared time; the same iterations once more with the overlap off give the
        # kernel's own duration (not timed for `value`)
        r = line["roofline"]
        dev.reset_stats()
        dev.set_option("timing", 1)
        dev.set_option("overlap_shadow", 0)
        dev.render_iterations(p, iters)
        si = dev.stats()
        dev.set_option("overlap_shadow", 1)
        dev.set_option("timing", 0)
        t_iso = si["ms_trace"] / 1e3 / max(1, si["launches_trace"])
        per_launch = r["algorithmic_bytes_per_launch"]
        r["isolated"] = {"avg_launch_us": round(t_iso * 1e6, 2),
                         "frac": round(per_launch / t_iso / 1e9 / HBM_PEAK_GBS, 4) if t_iso > 0 else None,
                         "frac_traffic": round(r["traffic"] / t_iso / 1e9 / HBM_PEAK_GBS, 4) if t_iso > 0 and r["traffic"] else None,
                         "note": "k_trace_refill alone (overlap_shadow 0): its own launch duration"}
        rp = load_rocprof(key, True)
        if rp:
            # the committed rocprofv3 profile of the same workload, also with overlap_shadow 0
            t = rp["avg_us"] * 1e-6
            r["isolated"]["rocprof"] = dict(rp, frac=round(per_launch / t / 1e9 / HBM_PEAK_GBS, 4),
                                            frac_traffic=round(r["traffic"] / t / 1e9 / HBM_PEAK_GBS, 4) if r["traffic"] else None)
        line["roofline_shadow"] = shadow_roofline(st, r["_inst"], si, key)
    elif isolated:
        def frame():
            dev.clear()
            dev.render_iterations(p, iters)
        isolated_extend(dev, frame, line["roofline"])
    line["roofline"].pop("_inst", None)
    line["roofline"].pop("_si", None)
    dev.close()
    del scene
    return line


class RankFrames:
    """One rank's frames of an N-GPU tile-sharded render: the
    film is cut into square tiles dealt round-robin to the ranks; a frame is
    every iteration of the rank's tiles, then igx_pack_tiles and one gather of
    the packed tiles to rank 0 (RCCL over xGMI), which assembles the frame.
    At N = 1 a frame is simply the whole film on one handle.

    N > 1: frames alternate between two device handles on the rank's GPU (own
    streams, framebuffer and path slots), so frame k+1's wavefront is queued
    before frame k is packed and gathered: the gather and frame k's tail
    kernel (its longest paths) overlap the next frame's
    bounces, as consecutive frames already overlap on one GPU (N = 1 has no
    per-frame synchronisation).  Every frame is fully rendered and gathered
    inside the timed region."""

    def __init__(self, ignis_amd, torch, dist, scene, W, H, spi, iters, rank, n, gpu, comm):
        from ignis_amd import shard
        self.ig, self.torch, self.dist, self.scene = ignis_amd, torch, dist, scene
        self.W, self.H, self.spi, self.iters, self.rank, self.n, self.gpu, self.comm = W, H, spi, iters, rank, n, gpu, comm
        self.tile = shard.balanced_tile(W, n)
        self.devs = [ignis_amd.Device(gpu)]
        self.devs[0].upload(scene)
        self.pending = []
        self.count = 0
        if n > 1:
            max_tiles = shard.max_tiles_per_rank(W, H, self.tile, n)
            self.pack = torch.zeros(max_tiles * self.tile * self.tile * 3, dtype=torch.float32, device="cuda")
            self.gather_bufs = [torch.zeros(self.pack.numel(), dtype=torch.float32, device=comm)
                                for _ in range(n)] if rank == 0 else None
            self.frame = torch.zeros((W * H, 3), dtype=torch.float32, device="cuda")
            dst = torch.from_numpy(shard.packed_destinations(W, H, self.tile, n)).cuda()
            self.valid = dst >= 0
            self.dst_valid = dst[self.valid]
            self.devs.append(ignis_amd.Device(gpu))
            self.devs[1].upload(scene)
            # one stream slot per handle when the rank's share of a frame is one
            # chunk (the other handle overlaps the next frame); a share of several
            # chunks keeps two, so consecutive chunks of a frame overlap as at N = 1
            for d in self.devs:
                d.set_option("stream_slots", rank_stream_slots(W, H, self.tile, n, spi, iters))
                d.set_option("slot_budget_mb", SLOT_BUDGET_MB if SLOT_BUDGET_MB or comm != "cpu"
                             else rehearsal_slot_budget_mb(torch, n))

    def params(self, it=0):
        p = self.ig.RenderParams()
        p.width, p.height, p.spi, p.iteration, p.frame, p.seed = self.W, self.H, self.spi, it, 0, 0
        if self.n > 1:
            p.tile_size, p.tile_offset, p.tile_stride = self.tile, self.rank, self.n
        return p

    def _pack(self, d):
        self.torch.cuda.current_stream().synchronize()  # the previous gather has read `pack`
        d.pack_tiles(self.params(0), self.pack.data_ptr(), self.pack.numel())  # waits for d's frame

    def _gather(self):
        # RCCL gather over xGMI to rank 0, assembled there
        self.dist.gather(self.pack if self.comm == "cuda" else self.pack.cpu(), self.gather_bufs, dst=0)
        if self.rank == 0:
            allpix = self.torch.cat(self.gather_bufs).to("cuda").view(-1, 3)
            self.frame[self.dst_valid] = allpix[self.valid]

    def render_frame(self):
        d = self.devs[self.count % len(self.devs)]
        self.count += 1
        d.clear()
        # all iterations of the frame in one call: iterations whose paths fit the
        # capacity are traced as one wavefront
        d.render_iterations(self.params(0), self.iters)
        if self.n > 1:
            # async_render: return once this frame's chunks are in their late
            # bounces, so the next frame (the other handle) overlaps only those
            d.wait_ready()
            if self.pending:
                e = self.pending.pop()
                self._pack(e)
                self._gather()
            self.pending.append(d)

    def drain(self):
        if self.pending:
            e = self.pending.pop()
            self._pack(e)
            self._gather()
        # igx_synchronize: the handle's worker thread (async_render) has queued
        # every frame and the GPU has finished them
        for d in self.devs:
            d.synchronize()
        self.torch.cuda.synchronize()

    def measure(self, steps, warmup):
        """warm-up, then `steps` frames between a barrier + synchronize on both
        sides; elapsed = the slowest rank's, ray totals summed over ranks"""
        torch, dist = self.torch, self.dist
        # every device handle renders (and gathers) at least once before timing:
        # its framebuffer, path slots and events are allocated outside the timed region
        for _ in range(max(warmup, len(self.devs))):
            self.render_frame()
        self.drain()
        for d in self.devs:
            d.reset_stats()
            d.set_option("timing", 1)
        if dist:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            self.render_frame()
        self.drain()
        if dist:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        st = self.devs[0].stats()
        for d in self.devs[1:]:
            s2 = d.stats()
            for key in ("camera_rays", "bounce_rays", "shadow_rays", "ms_trace", "ms_extend", "ms_shadow", "ms_finish",
                        "ms_generate", "ms_resolve", "launches_extend", "launches_trace", "extend_rays",
                        "extend_paths_out", "tail_shadow_rays", "tail_bounce_rays"):
                st[key] += s2[key]
        for d in self.devs:
            d.set_option("timing", 0)
        self.rank_rays = st["camera_rays"] + st["bounce_rays"] + st["shadow_rays"]
        totals = np.array([self.rank_rays, st["camera_rays"], st["bounce_rays"], st["shadow_rays"]], dtype=np.float64)
        if dist:
            t = torch.tensor([elapsed], dtype=torch.float64, device=self.comm)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())
            tt = torch.tensor(totals, dtype=torch.float64, device=self.comm)
            dist.all_reduce(tt, op=dist.ReduceOp.SUM)
            totals = tt.cpu().numpy()
        return {"elapsed": elapsed, "stats": st, "totals": totals,
                "slot_bytes": [int(d.stats()["slot_bytes"]) for d in self.devs]}

    def breakdown(self):
        """One more frame, untimed for `value`, by phase on every rank: render
        (all iterations of the rank's tiles, to completion), pack, then -- after
        a barrier, so no rank's wait for a slower one is counted -- the gather
        and rank 0's assembly; plus the rays of the rank's share in the timed
        frames.  Per-rank lists, min / max / mean (shard.rank_summary)."""
        from ignis_amd import shard
        torch, dist, d = self.torch, self.dist, self.devs[0]
        d.clear()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        d.render_iterations(self.params(0), self.iters)
        d.synchronize()
        t1 = time.perf_counter()
        self._pack(d)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        dist.barrier()
        t3 = time.perf_counter()
        self._gather()
        torch.cuda.synchronize()
        t4 = time.perf_counter()
        s = shard.rank_summary(dist, {"frame_ms": (t1 - t0) * 1e3, "pack_ms": (t2 - t1) * 1e3,
                                      "gather_ms": (t4 - t3) * 1e3, "mrays": self.rank_rays / 1e6},
                               "cpu" if self.comm == "cpu" else "cuda")
        f = s["frame_ms"]
        s["imbalance"] = round(f["max"] / f["min"], 4) if f["min"] > 0 else None
        s["note"] = ("frame_ms: one rank's tiles rendered alone (all iterations, to completion); pack_ms: "
                     "igx_pack_tiles; gather_ms: the gather to rank 0 after a barrier, plus rank 0's assembly; "
                     "mrays: the rank's rays over the timed frames")
        return s

    def check(self):
        """rank 0 renders the whole frame alone and compares the gathered frame
        of the last frame with it bit for bit (tile sharding is exact: DESIGN.md §6)"""
        torch, dist = self.torch, self.dist
        gathered = self.frame.cpu().numpy()
        ok = torch.tensor([0.0], dtype=torch.float64, device=self.comm)
        if self.rank == 0:
            ref = self.ig.Device(self.gpu)
            ref.upload(self.scene)
            p = self.ig.RenderParams()
            p.width, p.height, p.spi = self.W, self.H, self.spi
            ref.render_iterations(p, self.iters)
            full, _ = ref.framebuffer(self.W * self.H * 3)
            ref.close()
            ok[0] = float(np.array_equal(full.reshape(-1, 3), gathered))
        dist.broadcast(ok, 0)
        return bool(ok.item())

    def close(self):
        for d in self.devs:
            d.close()
        self.devs = []


def sharded_line(ignis_amd, torch, dist, path, size, spi, spp, rank, n, gpu, comm, steps, check):
    """A second multi-GPU line (BASELINE config 5's stand-in): the scene at a
    size x size film, `spp` samples, tile-sharded over the N ranks exactly as
    the headline frame, with the per-rank breakdown and the bit-exact check."""
    scene = ignis_amd.Scene.from_file(path)
    iters = max(1, math.ceil(spp / spi))
    # pre-flight before any collective of the line: every handle of every rank
    # renders its share once (allocating its buffers), and the ranks agree that
    # all did -- a rank failing here (e.g. out of memory) must not leave the
    # others waiting in a gather or barrier it never reaches
    rf, err = None, None
    try:
        rf = RankFrames(ignis_amd, torch, dist, scene, size, size, spi, iters, rank, n, gpu, comm)
        for d in rf.devs:
            d.clear()
            d.render_iterations(rf.params(0), iters)
            d.synchronize()
    except Exception as e:
        err = f"rank {rank}: {type(e).__name__}: {e}"
    if dist:
        flag = torch.tensor([1.0 if err else 0.0], dtype=torch.float64, device=comm)
        dist.all_reduce(flag, op=dist.ReduceOp.MAX)
        failed = flag.item() > 0
    else:
        failed = err is not None
    if failed:
        if rf is not None:
            rf.close()
        return {"error": err or "another rank failed its pre-flight frame"}
    m = rf.measure(steps, 1)
    line = {"workload": f"{os.path.basename(path)} {size}x{size}, {iters * spi} spp = {iters} iterations x spi {spi}, "
                        "path tracer, seed 0 (BASELINE config 5 stand-in, SURVEY.md §8d)",
            "scene": os.path.basename(path), "width": size, "height": size, "spp": iters * spi, "n_gpus": n,
            "steps": steps, "value": round(float(m["totals"][0]) / m["elapsed"] / 1e6, 2), "unit": "Mrays/s",
            "ms_per_step": round(m["elapsed"] / steps * 1e3, 3), "scaling": "strong",
            "tile": rf.tile if n > 1 else None}
    if n > 1:
        line["ranks"] = rf.breakdown()
        if check:
            line["frame_equals_single_gpu"] = rf.check()
    rf.close()
    return line


def launch_ranks(args):
    """`bench.py --gpus N` (N > 1) started without a launcher: run N ranks as a
    child `torch.distributed.run` (one process per GPU, rendezvous on
    127.0.0.1) with the same arguments, relay its output (rank 0 prints the
    JSON line) and return its exit code.  Runs before anything touches the
    GPU, and starts a child instead of replacing this process."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd).returncode


def main():
    args = parse()
    if args.gpus < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}: launch one rank per GPU "
                         f"(torch.distributed.run --nproc-per-node {args.gpus}) or drop the launcher")
    if os.environ.get("IGX_BENCH_LAUNCH_PROBE") == "1":
        # launcher test hook (tests/test_bench_launch.py): report the rank layout, touch no GPU
        # one write(2) of the whole line: the ranks share the pipe, and a line
        # written in pieces can interleave with another rank's
        sys.stdout.flush()
        os.write(sys.stdout.fileno(), (json.dumps({"rank": int(os.environ.get("RANK", "0")), "world": world,
                                                   "gpus": args.gpus}) + "\n").encode())
        return None
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    n_gpus = max(world, 1)

    import torch
    # IGX_BENCH_REHEARSAL=1: every rank on GPU 0, gloo with host staging -- a
    # one-GPU dry run of the multi-GPU path (tile sharding, pack, gather,
    # assembly, max-over-ranks timing); the real run uses RCCL, one GPU per rank
    rehearsal = os.environ.get("IGX_BENCH_REHEARSAL") == "1"
    gpu = 0 if (rehearsal or world == 1) else local_rank
    comm = "cpu" if rehearsal else "cuda"
    dist = None
    torch.cuda.set_device(gpu)
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo" if rehearsal else "nccl", init_method="env://")

    import ignis_amd

    scene = ignis_amd.Scene.from_file(args.scene)
    W, H = (args.size, args.size) if args.size > 0 else scene.film_size
    spi = args.spi
    iters = max(1, math.ceil(args.spp / spi))
    rf = RankFrames(ignis_amd, torch, dist, scene, W, H, spi, iters, rank, n_gpus, gpu, comm)
    dev, tile = rf.devs[0], rf.tile
    params = rf.params
    m = rf.measure(args.steps, args.warmup)
    elapsed, st, totals = m["elapsed"], m["stats"], m["totals"]
    ranks = rf.breakdown() if n_gpus > 1 else None
    frame_check = rf.check() if n_gpus > 1 and not args.no_check_frame else None

    # ---- roofline of the dominant kernel, live HIP-event timing ----
    scene_key = os.path.splitext(os.path.basename(args.scene))[0]
    roof = roofline(dev, st, lambda: dev.render(params(0)), n_gpus, scene_key)
    inst = roof.pop("_inst", None)
    roof_shadow = None
    if args.isolated and st["launches_trace"] == 0:
        def frame():
            dev.clear()
            dev.render_iterations(params(0), iters)
        isolated_extend(dev, frame, roof)
        si = roof.pop("_si")
        if n_gpus == 1 and si["launches_shadow"] > 0:
            roof_shadow = fused_shadow_roofline(st, inst, si, scene_key)
    roof["note"] = ("achieved counts the HBM bytes the kernel must move (path / radiance / shadow-ray streams; "
                    "table reads too when the tables exceed the Infinity Cache); traffic is the rocprofv3 PMC "
                    "measurement of the same kernel and workload; memory_system_gbs counts every table read "
                    "including LDS / cache hits (a work rate)")

    result = None
    if rank == 0:
        total_rays = float(totals[0])
        value = total_rays / elapsed / 1e6
        samples = float(W * H * iters * spi * args.steps)
        cpu = None
        parity = None
        if n_gpus == 1 and not args.no_cpu_baseline:
            cpu, parity = cpu_baseline(scene, dev, W, H, spi, args.cpu_seconds)
        suite = None
        if n_gpus == 1 and args.suite:
            # other scenes of SURVEY.md §8d, incl. the HBM roofline scene of record (S-soup-16M)
            suite = [suite_line(ignis_amd, 0, os.path.join(ROOT, "scenes", f), spi, n, size, bool(args.isolated))
                     for f, n, size in (("primitives.json", 8, None),
                                        # config 4 stand-in at its stated 1024 spp (128 iterations x spi 8)
                                        ("s_deep.json", 128, None), ("s_soup_1m.json", 2, None),
                                        ("s_soup_16m.json", 1, None),
                                        # config 5 stand-in: S-deep at 4096x4096, 64 spp
                                        ("s_deep.json", 8, (4096, 4096)))]
            for line in suite:
                r = line["roofline"]
                r["note"] = (
                    "HBM roofline scene of record: 1.8 GB of BVH + triangles, far above the on-chip caches"
                    if line["scene"] == "s_soup_16m.json" else
                    "tables fit half the 256 MB Infinity Cache: achieved counts the ray streams only"
                    if r["tables_on_chip"] else
                    "tables exceed half the Infinity Cache: achieved counts every table read as HBM traffic")
        result = {
            "metric": "Mrays/s (primary+secondary) at fixed spp; per-pixel L2 vs CPU ref",
            "value": round(value, 2),
            "unit": "Mrays/s",
            "n_gpus": n_gpus,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": f"synthetic camera paths over {os.path.basename(args.scene)} (scene data from the reference checkout or the SURVEY.md §8d generators)",
            "config": {
                "workload": f"{os.path.basename(args.scene)} {W}x{H}, {iters * spi} spp = {iters} iterations x spi {spi}, path tracer max_depth {scene.desc.technique.max_depth}, seed 0",
                "scene": os.path.basename(args.scene),
                "width": W, "height": H, "spp": iters * spi, "spi": spi,
                "parallelism": (f"tile-shard x{n_gpus} ({tile}x{tile} tiles round-robin) + "
                                + ("gloo (rehearsal: every rank on GPU 0)" if rehearsal else "RCCL gather to rank 0"))
                if n_gpus > 1 else "single GPU",
            },
            "msamples_per_s": round(samples / elapsed / 1e6, 2),
            "rays": {"camera": int(totals[1]), "bounce": int(totals[2]), "shadow": int(totals[3])},
            "kernel_ms": {"trace": round(st["ms_trace"], 3), "extend": round(st["ms_extend"], 3), "shadow": round(st["ms_shadow"], 3),
                          "finish": round(st["ms_finish"], 3),
                          "generate": round(st["ms_generate"], 3), "resolve": round(st["ms_resolve"], 3)},
            "roofline": roof,
            "roofline_shadow": roof_shadow,
            "cpu_baseline": cpu,
            "parity": parity,
            "suite": suite,
        }
        if frame_check is not None:
            result["frame_equals_single_gpu"] = frame_check
        if ranks is not None:
            result["ranks"] = ranks
        result["slot_bytes_per_handle"] = m["slot_bytes"]
        result["backend"] = ("gloo (rehearsal)" if rehearsal else "nccl (RCCL)") if n_gpus > 1 else None
    rf.close()
    if args.config5:
        # BASELINE config 5 stand-in (S-deep at 4096x4096, 64 spp),
        # measured the same way at every N: tile-sharded over the ranks, gathered
        # to rank 0, per-rank breakdown (the headline frame above is config 2)
        try:
            c5 = sharded_line(ignis_amd, torch, dist, os.path.join(ROOT, "scenes", "s_deep.json"), 4096, spi, 64, rank,
                              n_gpus, gpu, comm, args.config5_steps, not args.no_check_frame)
        except Exception as e:  # the headline line still prints
            c5 = {"error": f"{type(e).__name__}: {e}"}
        if result is not None:
            result["config5"] = c5
    if result is not None:
        print(json.dumps(result), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()
    return result


def cgroup_cpu_quota():
    """CPUs' worth of time the cgroup grants this process (cgroup v2 cpu.max,
    or v1 cfs quota / period), None when unlimited."""
    for path, split in (("/sys/fs/cgroup/cpu.max", None),
                        ("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", "/sys/fs/cgroup/cpu/cpu.cfs_period_us")):
        try:
            if split is None:
                q, per = open(path).read().split()[:2]
            else:
                q, per = open(path).read().strip(), open(split).read().strip()
            if q in ("max", "-1"):
                return None
            return max(1, int(math.ceil(int(q) / int(per))))
        except (OSError, ValueError):
            continue
    return None


def cpu_threads():
    """Threads of the CPU baseline.  The reference CPU device runs TBB with
    hardware_concurrency threads (Device.cpp:347), which counts the CPUs the
    process may run on (affinity) and ignores OMP_NUM_THREADS; so does this.
    The GPU boxes grant the job a cgroup CPU quota (cpu.max 1600000/100000 =
    16 CPUs) on a 256-CPU affinity mask: more threads than the quota are
    throttled to the same CPU time, so the baseline runs min(affinity, quota)
    threads and reports both numbers.  Returns (threads, affinity, quota)."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = cgroup_cpu_quota()
    return max(1, min(aff, quota) if quota else aff), aff, quota


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(scene, dev, W, H, spi, target_s):
    """Oracle (C restatement of the reference CPU device: binned-SAH BVH4 over
    Tri4 leaves, the device's wavefront loop per 16x16 tile -- cpu_trace,
    driver/mapping_cpu.art:694-836: a stream of spi * 256 rays, closest hits,
    sort by entity, shading, compaction, any-hit shadow stream) timed on this
    host with scripts/benchmark.sh's protocol (lines 13-14, 58-91): 2 warm-up
    runs, then 10 timed runs, min / median / max.  One run renders one
    iteration (spi samples) of a band of rows of the same frame, the band sized
    so that the 12 runs take about target_s; value = the median run.  Also the
    per-pixel parity of the GPU band (iteration 0)."""
    from oracle import oracle_py as O
    threads, affinity, quota = cpu_threads()
    orc = O.OracleScene(scene)
    # calibrate on 8 rows, then size the band for ~target_s / 12 per run
    y0 = H // 2
    _, st = orc.render(W, H, spi, iteration=0, threads=threads, window=(0, y0, W, y0 + 8), stream=True)
    rows = int(max(8, min(H, 8 * (target_s / 12) / max(st["seconds"], 1e-4))))
    y0 = max(0, H // 2 - rows // 2)
    win = (0, y0, W, y0 + rows)
    fb0 = None
    runs = []
    for it in range(12):
        fb, st = orc.render(W, H, spi, iteration=it, threads=threads, window=win, stream=True)
        if it == 0:
            fb0 = fb.copy()  # iteration 0, for the parity check below
        if it >= 2:  # 2 warm-up runs
            runs.append(((st["camera_rays"] + st["bounce_rays"] + st["shadow_rays"]) / st["seconds"] / 1e6, st["seconds"]))
    rates = sorted(r for r, _ in runs)
    med = float(np.median(rates))
    # the reference's TBB thread count as such (hardware_concurrency, Device.cpp:347),
    # measured beside the quota-sized run: 1 warm-up + 3 timed runs of the same band
    at_hc = None
    if affinity != threads:
        hc = []
        for it in range(4):
            _, st = orc.render(W, H, spi, iteration=it, threads=affinity, window=win, stream=True)
            if it >= 1:
                hc.append((st["camera_rays"] + st["bounce_rays"] + st["shadow_rays"]) / st["seconds"] / 1e6)
        at_hc = {"threads": affinity, "value": round(float(np.median(hc)), 3),
                 "note": "same band at the reference CPU device's thread count (TBB hardware_concurrency); "
                         "more threads than the cgroup CPU quota are throttled"}
    cpu = {
        "value": round(med, 3),
        "unit": "Mrays/s",
        "cores": threads,
        "kind": "port",
        "min_med_max": [round(rates[0], 3), round(med, 3), round(rates[-1], 3)],
        "per_thread": round(med / threads, 3),
        "cpu_model": cpu_model(),
        "machine_logical_cpus": os.cpu_count(),
        "hardware_concurrency": affinity,
        "cgroup_cpu_quota": quota,
        "at_hardware_concurrency": at_hc,
        "sample": f"oracle/oracle.c (restated reference CPU device: SAH BVH4 + Tri4 leaves, cpu_trace's wavefront of "
                  f"spi x 256 rays per 16x16 tile with sort by entity and compaction), {threads} threads "
                  f"(hardware_concurrency {affinity} on a {cpu_model()} host, cgroup CPU quota "
                  f"{quota if quota else 'none'}: min of the two), rows {y0}-{y0 + rows} of the "
                  f"{W}x{H} frame, 2 warm-up + 10 timed runs of one iteration (spi {spi}) each, "
                  f"{sum(t for _, t in runs):.1f} s timed",
    }
    # parity: GPU iteration 0 of the same frame vs the oracle band
    dev.clear()
    p = __import__("ignis_amd").RenderParams()
    p.width, p.height, p.spi = W, H, spi
    dev.render(p)
    g, _ = dev.framebuffer(W * H * 3)
    g = g.reshape(H, W, 3)[y0:y0 + rows]
    o = fb0.reshape(H, W, 3)[y0:y0 + rows]
    # RunEvaluations' error_image (scripts/RunEvaluations.py:80-87): RelSE where the
    # oracle pixel is non-zero, AbsSE where it is zero, clamped at the 99th percentile
    nz = o != 0
    e = np.where(nz, np.square((g - o) / np.where(nz, o, 1)), np.square(g))
    e = np.minimum(e, np.percentile(e, 99))
    parity = {
        "rows": [y0, y0 + rows],
        "pixel_l2_rmse": float(np.sqrt(np.mean((g - o) ** 2))),
        "rel_mse": float(e.mean()),
        "frac_pixels_rel_1e-2": float(np.mean(np.abs(g - o) <= 1e-2 * np.maximum(np.abs(o), 1e-2))),
        "mean_gpu": float(g.mean()), "mean_cpu": float(o.mean()),
    }
    return cpu, parity


if __name__ == "__main__":
    main()
