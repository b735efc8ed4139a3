"""Turn rocprofv3 CSV output under gpurun_out/ into the committed summaries
under profiles/ (kernel stats table; per-launch HBM traffic of k_extend).

FETCH_SIZE / WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half the
bytes of a wide read (MI355X_MICROARCH.md §HBM), so
hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024, per dispatch, averaged over
the k_extend dispatches of the counter pass.
"""
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def find(d, pattern):
    hits = sorted(glob.glob(os.path.join(d, "**", pattern), recursive=True))
    return hits[-1] if hits else None


def short(name):
    n = name.replace("(anonymous namespace)::", "")
    if n.startswith("void "):
        n = n[5:]
    return n.split("(")[0]


def second_half_stats(trace_csv):
    """rocprofv3 kernel stats rebuilt from the per-dispatch trace over the
    second half of each kernel's dispatches: tools/pmc_run.py renders twice
    (a warm-up of the same shape, then the measured render), so that half is
    the measured render alone."""
    by = {}
    for r in csv.DictReader(open(trace_csv)):
        by.setdefault(r["Kernel_Name"], []).append((int(r["Dispatch_Id"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    rows = []
    for name, ds in by.items():
        ds.sort()
        d = [t for _, t in ds[len(ds) // 2:]]
        if d:
            rows.append({"Name": name, "Calls": len(d), "TotalDurationNs": sum(d), "AverageNs": sum(d) / len(d),
                         "MinNs": min(d), "MaxNs": max(d)})
    total = sum(r["TotalDurationNs"] for r in rows) or 1
    for r in rows:
        r["Percentage"] = 100.0 * r["TotalDurationNs"] / total
    rows.sort(key=lambda r: -r["TotalDurationNs"])
    return rows


def kernel_stats(src_dir, tag, second_half=False):
    f = find(src_dir, "*kernel_trace.csv" if second_half else "*kernel_stats.csv")
    if not f:
        print("no kernel stats under", src_dir)
        return
    dst = os.path.join(ROOT, "profiles", f"{tag}_kernel_stats.csv")
    if second_half:
        rows = second_half_stats(f)
        with open(dst, "w", newline="") as o:
            w = csv.DictWriter(o, fieldnames=["Name", "Calls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs", "Percentage"])
            w.writeheader()
            w.writerows(rows)
    else:
        shutil.copy(f, dst)
        rows = list(csv.DictReader(open(f)))
    lines = [f"# rocprofv3 --kernel-trace --stats ({tag})" +
             (": the measured render, second half of each kernel's dispatches (tools/pmc_run.py warms up first)"
              if second_half else ""), "",
             "| kernel | calls | total ms | avg us | min us | max us | % |", "|---|---|---|---|---|---|---|"]
    for r in rows:
        lines.append(f"| `{short(r['Name'])}` | {r['Calls']} | {float(r['TotalDurationNs']) / 1e6:.3f} | "
                     f"{float(r['AverageNs']) / 1e3:.2f} | {float(r['MinNs']) / 1e3:.2f} | {float(r['MaxNs']) / 1e3:.2f} | "
                     f"{float(r['Percentage']):.2f} |")
    open(os.path.join(ROOT, "profiles", f"{tag}_kernel_stats.md"), "w").write("\n".join(lines) + "\n")
    print("\n".join(lines[:14]))


def pmc_file(kernel, scene):
    """profiles/pmc_<kernel>[_<scene>].json (bench.py's load_pmc reads the same name)."""
    k = kernel[2:] if kernel.startswith("k_") else kernel
    k = k.rstrip("<")
    return f"pmc_{k}.json" if scene == "diamond_scene" else f"pmc_{k}_{scene}.json"


def pmc(fetch_dir, write_dir, kernel="k_extend", scene="diamond_scene", workload=None, second_half=False):
    def per_dispatch(d, counter):
        f = find(d, "*counter_collection.csv")
        if not f:
            return {}
        out = {}
        for r in csv.DictReader(open(f)):
            if kernel in r["Kernel_Name"] and r["Counter_Name"] == counter:
                key = int(r.get("Dispatch_Id") or r.get("Correlation_Id"))
                out[key] = out.get(key, 0.0) + float(r["Counter_Value"])
        if second_half:  # the measured render (tools/pmc_run.py warms up first)
            keys = sorted(out)
            out = {k: out[k] for k in keys[len(keys) // 2:]}
        return out
    fs = per_dispatch(fetch_dir, "FETCH_SIZE")
    ws = per_dispatch(write_dir, "WRITE_SIZE")
    if not fs or not ws:
        print("missing counter data", len(fs), len(ws))
        return
    fetch = sum(fs.values()) / len(fs)
    write = sum(ws.values()) / len(ws)
    res = {
        "kernel": kernel,
        "workload": workload or f"tools/pmc_run.py: {scene}.json 1000x1000, spi 8 (the bench's iterations)",
        "dispatches_fetch_pass": len(fs), "dispatches_write_pass": len(ws),
        "fetch_size_kib_per_launch": round(fetch, 1),
        "write_size_kib_per_launch": round(write, 1),
        "hbm_bytes_per_launch": round((2 * fetch + write) * 1024, 1),
        "correction": "hbm = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE reports half of wide reads; MI355X_MICROARCH.md HBM section); Infinity-Cache hits are included in the counters",
    }
    name = pmc_file(kernel, scene)
    json.dump(res, open(os.path.join(ROOT, "profiles", name), "w"), indent=1)
    print(json.dumps(res, indent=1))


def calibration(fetch_dir, write_dir, trace_dir, log, tag):
    """FETCH_SIZE / WRITE_SIZE against known byte counts (tools/pmc_calibrate.hip):
    counter bytes per useful byte for each access pattern of the hot path."""
    def per_kernel(d, counter):
        f = find(d, "*counter_collection.csv")
        out = {}
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter:
                k = short(r["Kernel_Name"])
                out[k] = out.get(k, 0.0) + float(r["Counter_Value"]) * 1024
        return out
    fetch = per_kernel(fetch_dir, "FETCH_SIZE")
    write = per_kernel(write_dir, "WRITE_SIZE")
    dur = {short(r["Name"]): float(r["AverageNs"]) for r in csv.DictReader(open(find(trace_dir, "*kernel_stats.csv")))}
    rows = []
    for line in open(log):
        line = line.strip()
        if not line.startswith("{"):
            continue
        d = json.loads(line)
        k = d["kernel"]
        key = [n for n in fetch if n.endswith(k.split("<")[0]) and (("<" not in k) or k.split("<")[1].split(">")[0] in n)]
        key = key[0] if key else k
        useful = d.get("expected_unique_bytes", d.get("bytes"))
        rec = {"kernel": k, "useful_bytes": useful, "fetch_size_bytes": fetch.get(key, 0.0),
               "write_size_bytes": write.get(key, 0.0), "avg_ns": dur.get(key)}
        if "record_bytes" in d:
            rec["record_bytes"] = d["record_bytes"]
            rec["lines_128B_per_record"] = round(rec["fetch_size_bytes"] / 64 / d["lanes"], 3)
        rec["fetch_over_useful"] = round(rec["fetch_size_bytes"] / useful, 4) if "write" not in k else None
        rec["write_over_useful"] = round(rec["write_size_bytes"] / useful, 4) if "write" in k else None
        rows.append(rec)
    res = {"what": "rocprofv3 FETCH_SIZE / WRITE_SIZE vs known bytes on gfx950 (tools/pmc_calibrate.hip)",
           "finding": "FETCH_SIZE counts 64 B per 128-B line fetched from the memory side, for streaming and for "
                      "scattered 16/48/64/128-B records alike: HBM line bytes = 2 x FETCH_SIZE; WRITE_SIZE is exact "
                      "for streaming stores",
           "kernels": rows}
    json.dump(res, open(os.path.join(ROOT, "profiles", f"{tag}_pmc_calibration.json"), "w"), indent=1)
    print(json.dumps(res, indent=1))


def suite(tag):
    """profiles for every suite line (tools/gpu_profile_suite.sh): rocprof kernel
    stats as profiles/<tag>_<key>_kernel_stats.{csv,md} and the dominant
    kernel's PMC traffic as profiles/pmc_<kernel>_<key>.json (bench.py load_pmc)."""
    out = os.path.join(ROOT, "gpurun_out")
    for d in sorted(glob.glob(os.path.join(out, "suite_*"))):
        key = os.path.basename(d)[len("suite_"):]
        f = find(os.path.join(d, "trace"), "*kernel_stats.csv")
        if not f:
            print("no trace for", key)
            continue
        kernel_stats(os.path.join(d, "trace"), f"{tag}_{key}", second_half=True)
        names = [short(r["Name"]) for r in csv.DictReader(open(f))]
        # split-schedule scenes: the persistent-lane closest-hit kernel dominates
        kernel = "k_trace" if any("k_trace" in n for n in names) else "k_extend"
        args = ""
        for line in open(os.path.join(out, "suite.log")) if os.path.exists(os.path.join(out, "suite.log")) else []:
            if line.startswith(f"== {key}:"):
                args = line.split(":", 1)[1].strip()
        for k in [kernel] + (["k_shadow_refill"] if kernel == "k_trace" else []):
            # split schedule: the any-hit kernel gets its own roofline too (bench.py shadow_roofline)
            pmc(os.path.join(d, "fetch"), os.path.join(d, "write"), kernel=k, scene=key, second_half=True,
                workload=f"tools/{args or 'pmc_run.py'} (the suite line's scene, film and iterations, spi 8; "
                         f"the measured render after a warm-up of the same shape); "
                         f"rocprof kernel stats: profiles/{tag}_{key}_kernel_stats.md")


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "suite":
        suite(sys.argv[2])
        sys.exit(0)
    tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
    out = os.path.join(ROOT, "gpurun_out")
    kernel_stats(os.path.join(out, "prof"), tag)
    if os.path.isdir(os.path.join(out, "prof_soup")):
        kernel_stats(os.path.join(out, "prof_soup"), tag + "_s_soup_16m")
    if os.path.isdir(os.path.join(out, "cal_fetch")):
        calibration(os.path.join(out, "cal_fetch"), os.path.join(out, "cal_write"), os.path.join(out, "cal_trace"),
                    os.path.join(out, "cal_fetch.log"), tag)
    # the headline's counter passes (tools/gpu_lib.sh gpu_pmc, tag headline)
    pf, pw = (os.path.join(out, f"pmc_headline_{k}") for k in ("fetch", "write"))
    if not os.path.isdir(pf):
        pf, pw = os.path.join(out, "pmc_fetch"), os.path.join(out, "pmc_write")
    pmc(pf, pw)
    # the fused schedule's any-hit kernel from the same counter passes (bench.py fused_shadow_roofline)
    pmc(pf, pw, kernel="k_shadow<")
    if os.path.isdir(os.path.join(out, "pmc_fetch_soup")):
        # global-table scenes run split: k_trace (persistent-lane k_trace_refill) is the dominant kernel
        pmc(os.path.join(out, "pmc_fetch_soup"), os.path.join(out, "pmc_write_soup"), kernel="k_trace", scene="s_soup_16m")
