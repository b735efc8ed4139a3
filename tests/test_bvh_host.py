"""Host BVH builders (CPU only): closest hits through the binned-SAH BVH2, the
spatial-split BVH and the reader of the reference's GPU BLAS layout
(bvh2_from_reference, Node2 + Tri1 trees with leaves of 4 and 40 triangles)
equal brute force on random rays (tests/native/bvh_check.cpp, compiled here
with g++ against host/bvh_build.cpp)."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HOST = os.path.join(ROOT, "ignis-masterthesis_amd", "host")


def test_bvh_builders_match_brute_force(tmp_path):
    exe = str(tmp_path / "bvh_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-pthread", "-I", HOST, os.path.join(ROOT, "tests", "native", "bvh_check.cpp"),
                    os.path.join(HOST, "bvh_build.cpp"), "-o", exe], check=True)
    out = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    print(out.stdout)
    assert out.returncode == 0, out.stdout + out.stderr
    lines = [l.split() for l in out.stdout.splitlines() if " refs " in l]
    assert len(lines) == 16
    assert {l[1] for l in lines} == {"bvh2", "sbvh", "ref4", "ref40"}
    # spatial splits engage on the thin triangles and lower their SAH cost
    sl = {l[1]: l for l in lines if l[0] == "slivers"}
    assert int(sl["sbvh"][3].split("/")[0]) > int(sl["bvh2"][3].split("/")[0])
    assert float(sl["sbvh"][7]) < float(sl["bvh2"][7])


def test_light_hierarchy_depth_guard(tmp_path):
    """A light tree deeper than the 32-bit left/right codes falls back to the
    flux CDF selector (tests/native/light_select_check.cpp, g++ against
    host/light_select.cpp)."""
    exe = str(tmp_path / "light_select_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", HOST, "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "native", "light_select_check.cpp"), os.path.join(HOST, "light_select.cpp"),
                    "-o", exe], check=True)
    out = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0 and out.stdout.strip().endswith("ok"), out.stdout + out.stderr


def test_quantised_nodes_are_conservative(tmp_path):
    """Quantised 4-wide nodes (quantize_bvh4): every decoded child box holds
    the exact one with half a quantum to spare, and the device's quantised slab
    test (octant-ordered, exit widened) accepts every ray the exact test
    accepts, from origins up to 1e6 node extents away (tests/native/quantize_check.cpp)."""
    exe = str(tmp_path / "quantize_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-pthread", "-I", HOST, os.path.join(ROOT, "tests", "native", "quantize_check.cpp"),
                    os.path.join(HOST, "bvh_build.cpp"), "-o", exe], check=True)
    out = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0 and out.stdout.strip().endswith("ok"), out.stdout + out.stderr
