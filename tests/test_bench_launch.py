"""bench.py's multi-GPU launch contract, on CPU (no GPU call): `bench.py --gpus N`
started without a launcher runs N ranks itself as a child torch.distributed.run,
and a launcher whose WORLD_SIZE disagrees with --gpus is refused.  The
IGX_BENCH_LAUNCH_PROBE hook makes every rank print its layout and exit before
anything touches the GPU."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _objects(text):
    """Every JSON object printed on stdout.  The ranks share one pipe, so two
    ranks' lines may interleave without a newline between them: decode the
    objects one after the other instead of line by line."""
    dec, out, i = json.JSONDecoder(), [], 0
    while True:
        i = text.find("{", i)
        if i < 0:
            return out
        obj, i = dec.raw_decode(text, i)
        out.append(obj)


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["IGX_BENCH_LAUNCH_PROBE"] = "1"
    env.update(kw)
    return env


def test_gpus_n_launches_n_ranks():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--steps", "1"], env=_env(), capture_output=True, text=True,
                       timeout=180)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = _objects(r.stdout)
    assert sorted(x["rank"] for x in lines) == [0, 1]
    assert all(x["world"] == 2 and x["gpus"] == 2 for x in lines)


def test_single_gpu_needs_no_launcher():
    r = subprocess.run([sys.executable, BENCH], env=_env(), capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = _objects(r.stdout)
    assert lines == [{"rank": 0, "world": 1, "gpus": 1}]


def test_world_size_mismatch_is_refused():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "4"], env=_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert "WORLD_SIZE=2 but --gpus 4" in r.stderr


def _bench_module():
    import importlib.util
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("bench_under_test", os.path.join(root, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_limiters_come_from_committed_counter_profiles():
    """Every `limiter` string of the bench line is derived from a committed
    round-6 SQ/TCC summary of the same workload (bench.py sq_limiter), and the
    fractions it prints recompute from that file."""
    b = _bench_module()
    for scene, kernel in [("diamond_scene", "k_extend"), ("diamond_scene", "k_shadow"), ("s_deep", "k_extend"),
                          ("s_soup_16m", "k_trace_refill"), ("s_soup_16m", "k_shadow_refill")]:
        text = b.sq_limiter(scene, kernel)
        name = b.SQ_PROFILES[scene]
        assert f"profiles/{name}" in text, text
        with open(os.path.join(os.path.dirname(b.__file__), "profiles", name)) as f:
            ks = json.load(f)["kernels"]
        v = next(v for k, v in ks.items() if k.split("<")[0] == kernel)
        c = v["counters"]
        assert abs(v["wait_any"] - c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"]) < 1e-3
        assert abs(v["l2_hit"] - c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c["TCC_MISS_sum"])) < 1e-3
        assert f"{v['wait_any']:.0%} waiting" in text
    assert "no SQ counter profile" in b.sq_limiter("primitives", "k_extend")
