"""Per-merge timeline of the pipelined exchange from a rocprofv3 kernel trace
(tools/prof_window.sh-style directory): for the merges between bench.py's two
k_window_mark launches, the median duration of every kernel of an iteration and the
median gap before it (launch order k_select, k_find, k_commit, k_export_head, the
collective, k_import_fixed).

usage: python tools/fx_timeline.py gpurun_out/<dir>"""
import csv
import statistics
import sys


def main(d):
    rows = list(csv.DictReader(open(f"{d}/trace/run_kernel_trace.csv")))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    short = lambda n: n.replace("(anonymous namespace)::", "").split("(")[0].split("::")[-1].split("<")[0]  # noqa: E731
    seq = [(short(r["Kernel_Name"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
    marks = [i for i, x in enumerate(seq) if x[0] == "k_window_mark"]
    if len(marks) >= 2:
        seq = seq[marks[-2] + 1:marks[-1]]
    its, cur = [], None
    prev_end = None
    for name, s, e in seq:
        if name == "k_select":
            cur = []
            its.append(cur)
        if cur is not None:
            cur.append((name, (e - s) / 1000, (s - prev_end) / 1000 if prev_end else 0.0))
        prev_end = e
    its = [it for it in its if it]
    order = []
    for it in its:
        for n, _, _ in it:
            if n not in order:
                order.append(n)
    print(f"{len(its)} iterations in the window")
    tot = []
    for n in order:
        durs = [x[1] for it in its for x in it if x[0] == n]
        gaps = [x[2] for it in its for x in it if x[0] == n]
        print(f"  {n:28s} calls {len(durs):4d}  median {statistics.median(durs):7.2f} us  gap before {statistics.median(gaps):6.2f} us")
    for it in its[1:]:
        tot.append(sum(x[1] + x[2] for x in it))
    if tot:
        print(f"  per merge (kernels + gaps): median {statistics.median(tot):.1f} us")


if __name__ == "__main__":
    main(sys.argv[1])
