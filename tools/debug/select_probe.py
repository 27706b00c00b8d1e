"""Per-merge k_select time against the hot-list state (tools/debug; GPU box).

Runs a corpus merge by merge with HIP-event timing of k_select and prints, per
window of merges, the mean select time with the mean hot-list length, theta and
tied keys (geobpe_debug_state)."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "pt-bpe_amd"))
from geobpe import synth  # noqa: E402
from geobpe.engine import GeoBPEEngine  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
merges = int(sys.argv[2]) if len(sys.argv) > 2 else 5000
corpus = synth.make_corpus(synth.make_lengths(n, 40, 560, seed=0), seed=0)
eng = GeoBPEEngine(corpus, 5, device=0, max_vocab=1 << 20)
eng.initialize()
eng.bin()
eng.set_profiling(True, only="select")
buf = (ctypes.c_int64 * 10)()
rows = []
prev_ms, prev_n = 0.0, 0
for i in range(merges):
    if eng.run(1) != 1:
        break
    ms, nl = eng.kernel_ms("select")
    eng.L.geobpe_debug_state(eng._ctx, buf, 10)
    rows.append((1000 * (ms - prev_ms), nl - prev_n, *list(buf)))
    prev_ms, prev_n = ms, nl
a = np.array(rows, dtype=np.float64)
W = max(1, len(a) // 20)
print("merges  select_us/merge  launches  list_len  theta  ties  maxc  nskip")
for s in range(0, len(a), W):
    w = a[s:s + W]
    print(f"{s:5d}  {w[:, 0].mean():8.2f}  {w[:, 1].mean():5.2f}  {w[:, 2].mean():9.0f}  {w[:, 3].mean():7.1f}"
          f"  {w[:, 4].mean():6.1f}  {w[:, 5].mean():7.0f}  {w[:, 6].max():5.0f}")
top = np.argsort(-a[:, 0])[:10]
print("slowest:", [(int(i), round(a[i, 0], 1), int(a[i, 2]), int(a[i, 4])) for i in top])
