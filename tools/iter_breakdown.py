"""Per-iteration-range kernel time breakdown of a tools/prof.sh trace (merge-loop
kernels in launch order; one iteration = the kernels from one k_mark to the next)."""
import csv
import statistics
import sys

LOOP = ("k_select", "k_mark", "k_apply")


def main(d):
    rows = list(csv.DictReader(open(f"{d}/trace/run_kernel_trace.csv")))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    short = lambda n: n.replace("(anonymous namespace)::", "").split("(")[0].split("::")[-1]  # noqa: E731
    seq = [(short(r["Kernel_Name"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000) for r in rows]
    seq = [x for x in seq if x[0] in LOOP]
    first = "k_select" if any(x[0] == "k_select" for x in seq) else "k_mark"
    its, cur = [], None
    for k, t in seq:
        if k == first:
            cur = {}
            its.append(cur)
        if cur is not None:
            cur[k] = cur.get(k, 0.0) + t
    names = [k for k in LOOP if any(k in it for it in its)]
    print(len(its), "iterations; total kernel ms", round(sum(sum(it.values()) for it in its) / 1000, 2))
    for a, b in [(0, 10), (10, 50), (50, 100), (100, 200), (200, 500), (500, len(its))]:
        s = its[a:b]
        print(f"{a}-{b}: ms " + " ".join(f"{k[2:]} {sum(x.get(k, 0) for x in s) / 1000:.2f}" for k in names))
    late = its[500:]
    print("late medians us", {k[2:]: round(statistics.median([x.get(k, 0) for x in late]), 2) for k in names})


if __name__ == "__main__":
    main(sys.argv[1])
