"""Phase timeline of k_apply for a few early merges on the C3 corpus
(geobpe_debug_timeline): per-workgroup wall-clock stamps (100 MHz)."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "pt-bpe_amd"))
import torch  # noqa: E402,F401
from geobpe import _native, synth  # noqa: E402
from geobpe.engine import GeoBPEEngine  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
iters = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "1,2,3,20,200,800").split(",")]
corpus = synth.make_corpus(synth.make_lengths(n, 40, 560, seed=0), seed=0)
eng = GeoBPEEngine(corpus, 5).initialize()
eng.bin()
L = _native.lib()
done = 0
for it in iters:
    eng.run(it - done - 1)
    done = it - 1
    m = L.geobpe_debug_timeline(eng._ctx, 1, None, 0)
    eng.run(1)
    done += 1
    buf = np.zeros(m, dtype=np.int64)
    L.geobpe_debug_timeline(eng._ctx, 0, buf.ctypes.data_as(ctypes.c_void_p), m)
    t = buf.reshape(-1, 64)
    t = t[(t > 0).any(axis=1)]
    if len(t) == 0:
        print(f"merge {it}: (rebuild iteration / no stamps)")
        continue
    base = t[:, 0][t[:, 0] > 0].min()
    rel = (t - base) / 100.0  # us
    rel[:, 63][t[:, 63] == 0] = np.nan
    rel[t == 0] = np.nan
    last = eng.merges[-1]
    print(f"merge {it}: count {last[1]} merged {last[2]}  workgroups {len(t)}")
    names = {0: "start", 1: "setup", 60: "loop_end", 61: "flush_end", 62: "klist_end", 63: "end",
             20: "SEL.start", 21: "SEL.scanned", 22: "SEL.max", 23: "SEL.ties", 24: "SEL.staged", 25: "SEL.tourn",
             26: "SEL.end", 10: "MARK.start", 11: "MARK.state", 12: "MARK.bucket", 13: "MARK.hits"}
    names.update({30: "r0.res.kc", 31: "r0.res.reprobe", 32: "r0.res.cas", 33: "r0.res.done", 34: "flush.issued", 35: "flush.returned", 36: "flush.hot"})
    for r in range(2):
        for i, nm in enumerate(["front.loads", "front.agg", "finL.kc", "finL.store", "finL.agg", "finR.kc",
                                "finR.store", "finR.agg"]):
            names[40 + 10 * r + i] = f"r{r}.{nm}"
    if not np.all(np.isnan(rel[:, 63])):
        order = np.argsort(-np.nan_to_num(rel[:, 63], nan=-1))[:5]
        print("  slowest workgroups (end):", [(int(np.flatnonzero((t > 0).any(axis=1))[i]) if False else int(i),
                                              round(float(rel[i, 63]), 1)) for i in order])
    for k in sorted(range(64), key=lambda k: np.nanmedian(rel[:, k]) if not np.all(np.isnan(rel[:, k])) else 0):
        col = rel[:, k]
        if np.all(np.isnan(col)):
            continue
        name = names.get(k, f"r{(k - 2) // 4}." + ["front", "resolve", "barrier", "finish"][(k - 2) % 4])
        print(f"  {name:14s} min {np.nanmin(col):8.1f}  med {np.nanmedian(col):8.1f}  max {np.nanmax(col):8.1f}")
eng.close()
