"""Per-iteration-range kernel time breakdown of a tools/prof.sh trace."""
import csv
import statistics
import sys


def main(d):
    rows = list(csv.DictReader(open(f"{d}/trace/run_kernel_trace.csv")))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    short = lambda n: n.replace("(anonymous namespace)::", "").split("(")[0].split("::")[-1]  # noqa: E731
    seq = [(short(r["Kernel_Name"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000) for r in rows]
    seq = [x for x in seq if x[0] in ("k_select", "k_mark", "k_apply")]
    its = [(seq[i][1], seq[i + 1][1], seq[i + 2][1]) for i in range(0, len(seq) - 2, 3)]
    print(len(its), "iterations; total kernel ms", round(sum(map(sum, its)) / 1000, 2))
    for a, b in [(0, 10), (10, 50), (50, 100), (100, 200), (200, 500), (500, len(its))]:
        s = its[a:b]
        print(f"{a}-{b}: ms select {sum(x[0] for x in s)/1000:.2f} mark {sum(x[1] for x in s)/1000:.2f} "
              f"apply {sum(x[2] for x in s)/1000:.2f}")
    late = its[500:]
    print("late medians us", [round(statistics.median([x[k] for x in late]), 2) for k in range(3)])


if __name__ == "__main__":
    main(sys.argv[1])
