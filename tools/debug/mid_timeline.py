"""Phase timeline of the middle-regime kernels (mid.h: k_mid_sel = select + the previous
merge's place, k_mid_find) for a few merges on the C3 corpus, all merges in the middle
regime (geobpe_debug_timeline: per-workgroup 100 MHz stamps, relative to the select's
first stamp).  usage: python tools/debug/mid_timeline.py [merge,merge,...] [mid]"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "pt-bpe_amd"))
import torch  # noqa: E402,F401
from geobpe import _native, synth  # noqa: E402
from geobpe.engine import GeoBPEEngine  # noqa: E402

iters = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "20,200,800").split(",")]
mid = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 30
corpus = synth.make_corpus(synth.make_lengths(100_000, 40, 560, seed=0), seed=0)
eng = GeoBPEEngine(corpus, 5, mid=mid, tail=0).initialize()
eng.bin()
L = _native.lib()
names = {10: "F.start", 11: "F.setup", 15: "F.walked", 16: "F.deduped", 17: "F.resolved", 12: "F.rounds", 13: "F.end",
         30: "A.start", 32: "A.counted", 33: "A.grown", 35: "A.end", 36: "P.start", 37: "P.end",
         20: "S.start", 21: "S.scanned", 22: "S.max", 23: "S.ties", 24: "S.staged", 25: "S.tourn", 26: "S.end"}
done = 0
for it in iters:
    eng.run(it - done - 1)
    done = it - 1
    m = L.geobpe_debug_timeline(eng._ctx, 1, None, 0)
    eng.run(1)
    done += 1
    eng.synchronize()
    buf = np.zeros(m, dtype=np.int64)
    L.geobpe_debug_timeline(eng._ctx, 0, buf.ctypes.data_as(ctypes.c_void_p), m)
    t = buf.reshape(-1, 64)
    t = t[(t > 0).any(axis=1)]
    if len(t) == 0:
        print(f"merge {it}: (no stamps)")
        continue
    base = t[:, 20][t[:, 20] > 0].min() if (t[:, 20] > 0).any() else t[t > 0].min()
    rel = (t - base) / 100.0
    rel[t == 0] = np.nan
    last = eng.merges[-1]
    print(f"merge {it}: count {last[1]} merged {last[2]}  rows {len(t)}")
    cols = [k for k in range(64) if not np.all(np.isnan(rel[:, k]))]
    for k in sorted(cols, key=lambda k: np.nanmedian(rel[:, k])):
        col = rel[:, k]
        print(f"  {names.get(k, str(k)):12s} min {np.nanmin(col):8.1f}  med {np.nanmedian(col):8.1f}  max {np.nanmax(col):8.1f}")
eng.close()
