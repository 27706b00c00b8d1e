"""Kernel-by-kernel summary of a rocprofv3 kernel trace of a bench.py run, restricted to the
timed window between bench.py's two k_window_mark launches: per-kernel count / average /
total, the idle time between consecutive dispatches and the largest gaps.
usage: python tools/trace_window.py <dir with *kernel_trace.csv>"""
import collections
import csv
import glob
import sys


def short(n):
    # (a template kernel demangles with its return type and arguments: "void gb::k_commit<false>(...)")
    n = n.replace("(anonymous namespace)::", "").replace("gb::", "").split("(")[0].split("::")[-1]
    return n.split("<")[0].split(" ")[-1]


f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if short(r["Kernel_Name"]) == "k_window_mark"]
w = rows[idx[0] + 1:idx[1]]
t0, t1 = int(rows[idx[0]]["End_Timestamp"]), int(rows[idx[1]]["Start_Timestamp"])
agg = collections.defaultdict(list)
for r in w:
    agg[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
print(f"window {(t1 - t0) / 1e3:.1f} us, {len(w)} dispatches")
for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    print(f"  {k:24s} n={len(v):4d} avg={sum(v) / len(v):8.2f} us  total={sum(v):9.1f} us")
prev, gaps = t0, []
for r in w:
    gaps.append(((int(r["Start_Timestamp"]) - prev) / 1e3, short(r["Kernel_Name"])))
    prev = int(r["End_Timestamp"])
gaps.append(((t1 - prev) / 1e3, "(end mark)"))
print(f"  idle {sum(g for g, _ in gaps):.1f} us; largest gaps (us, before): {[(round(g, 1), k) for g, k in sorted(gaps, reverse=True)[:6]]}")
