"""Summarise a tools/prof.sh output dir: per-kernel stats, per-iteration profile
and PMC FETCH/WRITE bytes per launch (gfx950: FETCH_SIZE counts half of wide
streaming reads -> x2, MI355X_MICROARCH.md §HBM)."""
import collections
import csv
import json
import sys


def short(n):
    return n.replace("(anonymous namespace)::", "").replace("gb::", "").split("(")[0]


def main(d):
    rows = list(csv.DictReader(open(f"{d}/trace/run_kernel_trace.csv")))
    by = collections.defaultdict(list)
    for r in rows:
        by[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
    out = {"trace": {}, "pmc": {}}
    for k, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
        if not k.startswith("k_"):
            continue
        n = len(v)
        q = sorted(v)
        out["trace"][k] = {"calls": n, "total_us": round(sum(v), 1), "avg_us": round(sum(v) / n, 2),
                           "p50_us": round(q[n // 2], 2), "max_us": round(q[-1], 1),
                           "first5": [round(x, 1) for x in v[:5]], "last3": [round(x, 1) for x in v[-3:]]}
    for c in ("fetch", "write"):
        try:
            rows = list(csv.DictReader(open(f"{d}/pmc_{c}/run_counter_collection.csv")))
        except FileNotFoundError:
            continue
        agg = collections.defaultdict(list)
        for r in rows:
            agg[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
        for k, v in agg.items():
            if k.startswith("k_"):
                out["pmc"].setdefault(k, {})[c + "_KB_avg"] = round(sum(v) / len(v), 1)
    # HBM bytes per launch: FETCH_SIZE (KB) counts half of wide streaming reads on gfx950 -> x2
    for k, v in out["pmc"].items():
        if "fetch_KB_avg" in v and "write_KB_avg" in v:
            v["hbm_bytes_per_launch"] = 1024.0 * (2 * v["fetch_KB_avg"] + v["write_KB_avg"])
    return out


if __name__ == "__main__":
    r = main(sys.argv[1])
    if len(sys.argv) > 2:  # write the bench's traffic source (profiles/pmc_latest.json)
        with open(sys.argv[2], "w") as f:
            json.dump({"source": sys.argv[3] if len(sys.argv) > 3 else sys.argv[1],
                       "note": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of the bench command; "
                               "hbm_bytes_per_launch = 1024 * (2 * FETCH_SIZE + WRITE_SIZE)",
                       "kernels": r["pmc"]}, f, indent=1)
    print(json.dumps(r, indent=1))
