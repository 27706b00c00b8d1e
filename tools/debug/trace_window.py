"""Per-kernel totals inside the bench's timed window (between the two k_window_mark
launches) of a rocprofv3 --kernel-trace database.  usage: trace_window.py <run_results.db>"""
import collections
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
rows = db.execute("select name, start, end from kernels order by start").fetchall()
w = [i for i, r in enumerate(rows) if "window_mark" in r[0]]
a, b = w[0], w[-1]
seg = rows[a:b + 1]
T = (seg[-1][1] - seg[0][2]) / 1e3
tot, cnt = collections.defaultdict(float), collections.Counter()
for r in seg[1:-1]:
    k = r[0].split("(")[0]
    tot[k] += (r[2] - r[1]) / 1e3
    cnt[k] += 1
busy = sum(tot.values())
print(f"window {T:.1f} us, kernels busy {busy:.1f} us ({busy / T:.1%})")
for k in sorted(tot, key=lambda k: -tot[k]):
    print(f"{k:40s} {cnt[k]:6d} {tot[k]:10.1f} us {tot[k] / cnt[k]:8.2f} us/launch")
