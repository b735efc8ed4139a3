"""Dev tool: idle time of the GPU in a rocprofv3 --kernel-trace CSV (union of
all dispatches' [start, end) intervals), over the last `frac` of the trace
(tools/chunk_probe.py renders a warm-up and two timed repetitions), with the
largest gaps and the kernels on either side.
usage: timeline_gaps.py kernel_trace.csv [frac=0.5] [top=15]"""
import csv
import sys

rows = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("void ", ""))
        for r in csv.DictReader(open(sys.argv[1]))]
frac = float(sys.argv[2]) if len(sys.argv) > 2 else 0.5
top = int(sys.argv[3]) if len(sys.argv) > 3 else 15
rows.sort()
t_end = max(e for _, e, _ in rows)
t0 = rows[0][0] + (t_end - rows[0][0]) * (1 - frac)
rows = [r for r in rows if r[0] >= t0]
busy, gaps, cur_s, cur_e, last = 0, [], rows[0][0], rows[0][1], rows[0][2]
for s, e, k in rows[1:]:
    if s > cur_e:
        busy += cur_e - cur_s
        gaps.append((s - cur_e, last, k, cur_e))
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
    if e >= cur_e:
        last = k
busy += cur_e - cur_s
span = rows[-1][1] - rows[0][0]
print(f"span {span / 1e6:.2f} ms, busy {busy / 1e6:.2f} ms, idle {(span - busy) / 1e6:.2f} ms in {len(gaps)} gaps")
for g, a, b, t in sorted(gaps, reverse=True)[:top]:
    print(f"  gap {g / 1e3:9.1f} us at {(t - rows[0][0]) / 1e6:8.2f} ms: after {a[:60]} -> before {b[:60]}")
