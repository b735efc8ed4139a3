"""Summary of tools/gpu_pmc_sq.sh's three counter passes: per kernel, summed
over the measured render's dispatches (the second half, as
tools/profile_summary.py: pmc_run.py renders a warm-up of the same shape
first), with unit-free ratios.  SQ_WAVE_CYCLES, SQ_WAIT_*, SQ_ACTIVE_INST_*
count in the same (quad-cycle) unit, and WAIT_ANY + WAIT_INST_ANY +
ACTIVE_INST_ANY ~ WAVE_CYCLES (MI355X_MICROARCH.md, rocprofv3 PMC slots), so
  wait_any          share of wave cycles parked on s_waitcnt (memory / LDS latency)
  wait_inst_any     share stalled at issue (dependency, pipe busy)
  active_inst_any   share issuing an instruction
  valu_active       share issuing VALU
  lane_util         SQ_THREAD_CYCLES_VALU / (64 * SQ_ACTIVE_INST_VALU): active lanes per VALU instruction
  l2_hit            TCC_HIT / (TCC_HIT + TCC_MISS)
usage: pmc_sq_summary.py gpurun_out/sq_TAG [out.json]"""
import collections
import csv
import glob
import json
import os
import sys


def kernel(name):
    n = name.replace("void ", "").replace("(anonymous namespace)::", "").replace("igxh::", "")
    return n.split("(")[0]


def passes(root):
    out = collections.defaultdict(lambda: collections.defaultdict(float))
    disp_total = {}
    for f in sorted(glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True)):
        per = collections.defaultdict(lambda: collections.defaultdict(float))
        for r in csv.DictReader(open(f)):
            per[(kernel(r["Kernel_Name"]), int(r["Dispatch_Id"]))][r["Counter_Name"]] += float(r["Counter_Value"])
        by_k = collections.defaultdict(list)
        for (k, d), c in per.items():
            by_k[k].append((d, c))
        for k, lst in by_k.items():
            lst.sort()
            keep = lst[len(lst) // 2:] if len(lst) > 1 else lst  # the measured render
            disp_total[k] = len(keep)
            for _, c in keep:
                for n, v in c.items():
                    out[k][n] += v
    return out, disp_total


def main():
    root = sys.argv[1]
    agg, disp = passes(root)
    res = {}
    for k, d in agg.items():
        if not k.startswith("k_") or "SQ_WAVE_CYCLES" not in d:
            continue
        wc = d["SQ_WAVE_CYCLES"]
        r = {"dispatches": disp[k], "counters": {n: v for n, v in sorted(d.items())}}
        r["wait_any"] = round(d.get("SQ_WAIT_ANY", 0) / wc, 3)
        r["wait_inst_any"] = round(d.get("SQ_WAIT_INST_ANY", 0) / wc, 3)
        r["active_inst_any"] = round(d.get("SQ_ACTIVE_INST_ANY", 0) / wc, 3)
        r["valu_active"] = round(d.get("SQ_ACTIVE_INST_VALU", 0) / wc, 3)
        if d.get("SQ_ACTIVE_INST_VALU"):
            r["lane_util"] = round(d.get("SQ_THREAD_CYCLES_VALU", 0) / (64 * d["SQ_ACTIVE_INST_VALU"]), 3)
        if d.get("SQ_WAVES"):
            r["valu_insts_per_wave"] = round(d.get("SQ_INSTS_VALU", 0) / d["SQ_WAVES"], 1)
            r["vmem_rd_per_wave"] = round(d.get("SQ_INSTS_VMEM_RD", 0) / d["SQ_WAVES"], 1)
            r["lds_insts_per_wave"] = round(d.get("SQ_INSTS_LDS", 0) / d["SQ_WAVES"], 1)
        if d.get("TCC_HIT_sum", 0) + d.get("TCC_MISS_sum", 0) > 0:
            r["l2_hit"] = round(d["TCC_HIT_sum"] / (d["TCC_HIT_sum"] + d["TCC_MISS_sum"]), 3)
        if d.get("SQ_LDS_IDX_ACTIVE"):
            r["lds_bank_conflict_share"] = round(d.get("SQ_LDS_BANK_CONFLICT", 0) / d["SQ_LDS_IDX_ACTIVE"], 3)
        res[k] = r
    txt = json.dumps({"source": root, "kernels": res}, indent=1)
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(txt + "\n")
    for k, r in sorted(res.items(), key=lambda kv: -kv[1]["counters"].get("SQ_WAVE_CYCLES", 0)):
        print(k, {n: v for n, v in r.items() if n != "counters"})


if __name__ == "__main__":
    main()
