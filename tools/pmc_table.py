"""Dev tool: per-kernel sums of a rocprofv3 counter CSV and derived ratios.
usage: pmc_table.py gpurun_out/valu/p1/run_counter_collection.csv [...]"""
import collections
import csv
import sys

CU = 256
for path in sys.argv[1:]:
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").replace("igxh::", "").split("(")[0]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
    for k, d in sorted(agg.items(), key=lambda kv: -kv[1].get("GRBM_GUI_ACTIVE", 0)):
        if not k.startswith("k_"):
            continue
        out = {c: f"{v:.4g}" for c, v in d.items()}
        g = d.get("GRBM_GUI_ACTIVE", 0) / 8  # summed over the 8 XCDs
        if "SQ_ACTIVE_INST_VALU" in d and g:
            out["VALUBusy%"] = f"{100 * d['SQ_ACTIVE_INST_VALU'] / CU / g:.1f}"
        if "SQ_THREAD_CYCLES_VALU" in d:
            out["VALUUtil%"] = f"{100 * d['SQ_THREAD_CYCLES_VALU'] / (d['SQ_ACTIVE_INST_VALU'] * 64):.1f}"
        if "SQ_WAVE_CYCLES" in d:
            out["wait_any/wave_cyc"] = f"{d['SQ_WAIT_INST_ANY'] / d['SQ_WAVE_CYCLES']:.2f}"
            out["valu/wave_cyc"] = f"{d['SQ_ACTIVE_INST_VALU'] / d['SQ_WAVE_CYCLES']:.2f}"
        if "TCC_HIT_sum" in d:
            out["L2hit"] = f"{d['TCC_HIT_sum'] / (d['TCC_HIT_sum'] + d['TCC_MISS_sum']):.2f}"
        print(f"{k} [{len(disp[k])} dispatches]: {out}")
