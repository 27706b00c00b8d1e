"""Per-kernel summary of a tools/prof_window.sh output dir, restricted to the
dispatches between bench.py's two k_window_mark launches (its timed region):
trace durations, and HBM bytes per launch from the FETCH_SIZE / WRITE_SIZE passes
(gfx950: FETCH_SIZE tallies 128-B requests at 64 B -> x2; MI355X_MICROARCH.md
§HBM).  The PMC passes run the same bench command, so the same window.

usage: python tools/prof_window.py <dir>            -> JSON on stdout
       python tools/prof_window.py <dir> --save <profiles/pmc_windows.json> <source>"""
import collections
import csv
import json
import os
import sys

MARK = "k_window_mark"


def short(n):
    # (a template kernel demangles with its return type and arguments: "void gb::k_commit<false>(...)")
    n = n.replace("(anonymous namespace)::", "").replace("gb::", "").split("(")[0].split("::")[-1]
    return n.split("<")[0].split(" ")[-1]


def _order(r):
    for k in ("Dispatch_Id", "Correlation_Id"):
        if k in r and r[k] not in ("", None):
            return int(r[k])
    return int(r["Start_Timestamp"])


def window(rows, pre=False):
    """rows (one per dispatch) strictly between the first two marker dispatches
    (pre: the rows before the first one -- the prologue and bin pass)."""
    rows = sorted(rows, key=_order)
    idx = [i for i, r in enumerate(rows) if short(r["Kernel_Name"]) == MARK]
    if len(idx) < 2:
        raise SystemExit(f"expected 2 {MARK} dispatches, found {len(idx)}")
    return rows[: idx[0]] if pre else rows[idx[0] + 1: idx[1]]


def main(d):
    out = {"trace": {}, "pmc": {}, "pre_pmc": {}}
    tr = window(list(csv.DictReader(open(f"{d}/trace/run_kernel_trace.csv"))))
    by = collections.defaultdict(list)
    for r in tr:
        by[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
    for k, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
        q = sorted(v)
        out["trace"][k] = {"calls": len(v), "total_us": round(sum(v), 2), "avg_us": round(sum(v) / len(v), 3),
                           "p50_us": round(q[len(q) // 2], 2), "min_us": round(q[0], 2), "max_us": round(q[-1], 2)}
    if tr:
        out["window_wall_us"] = round((int(tr[-1]["End_Timestamp"]) - int(tr[0]["Start_Timestamp"])) / 1000, 2)
        # the GPU's idle time inside the window: the gaps between consecutive dispatches (host
        # waits, allocations, launch latency), by the kernel pair around them
        gaps, by_pair = [], collections.defaultdict(list)
        t = sorted(tr, key=lambda r: int(r["Start_Timestamp"]))
        end = int(t[0]["End_Timestamp"])
        for a, b in zip(t, t[1:]):
            g = (int(b["Start_Timestamp"]) - end) / 1000
            end = max(end, int(b["End_Timestamp"]))
            if g > 0:
                gaps.append((g, short(a["Kernel_Name"]), short(b["Kernel_Name"])))
                by_pair[short(a["Kernel_Name"]) + " -> " + short(b["Kernel_Name"])].append(g)
        out["idle"] = {"total_us": round(sum(g for g, _, _ in gaps), 2),
                       "by_pair": {k: {"n": len(v), "total_us": round(sum(v), 2), "max_us": round(max(v), 2)}
                                   for k, v in sorted(by_pair.items(), key=lambda kv: -sum(kv[1]))[:12]},
                       "largest": [[round(g, 2), a, b] for g, a, b in sorted(gaps, reverse=True)[:12]]}
    for c, name in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
        p = f"{d}/pmc_{c}/run_counter_collection.csv"
        if not os.path.exists(p):
            continue
        rows = [r for r in csv.DictReader(open(p)) if r.get("Counter_Name", name) == name]
        for part, pre in (("pmc", False), ("pre_pmc", True)):
            agg = collections.defaultdict(list)
            for r in window(rows, pre):
                agg[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
            for k, v in agg.items():
                out[part].setdefault(k, {})[c + "_KB_avg"] = round(sum(v) / len(v), 2)
                out[part][k][c + "_launches"] = len(v)
    for part in ("pmc", "pre_pmc"):
        for k, v in out[part].items():
            if "fetch_KB_avg" in v and "write_KB_avg" in v:
                v["hbm_bytes_per_launch"] = round(1024.0 * (2 * v["fetch_KB_avg"] + v["write_KB_avg"]), 1)
    return out


if __name__ == "__main__":
    r = main(sys.argv[1])
    if len(sys.argv) > 3 and sys.argv[2] == "--save":
        path, src = sys.argv[3], sys.argv[4]
        args = open(os.path.join(sys.argv[1], "bench_args.txt")).read().split()
        get = lambda f, dflt: args[args.index(f) + 1] if f in args else dflt  # noqa: E731
        key = f"config={get('--config', 'c3')},warmup={get('--warmup', '10')},steps={get('--steps', '990')},n=1"
        db = json.load(open(path)) if os.path.exists(path) else {}
        db[key] = {"source": src, "note": "dispatches between bench.py's k_window_mark launches; "
                   "hbm_bytes_per_launch = 1024 * (2 * FETCH_SIZE + WRITE_SIZE)", "kernels": r["pmc"],
                   "pre_kernels": r["pre_pmc"],
                   "trace": r["trace"]}
        json.dump(db, open(path, "w"), indent=1, sort_keys=True)
    print(json.dumps(r, indent=1))
