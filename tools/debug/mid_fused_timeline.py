"""Phase timeline of the fused middle-regime find launch (k_mid_find of merge t+1: its find
workgroups 0..G-1 and, beside them, the appending workgroups G..G+31 that write merge t's
posting entries) on the C3 corpus: per-workgroup 100 MHz stamps relative to the launch's
first find stamp, find and append rows kept apart (the flush after the run writes its own
append stamps to rows 0..31, which are ignored here).
usage: python tools/debug/mid_fused_timeline.py [merge,merge,...]"""
import ctypes
import os
import sys

os.environ.setdefault("GEOBPE_SPEC", "0")  # (no idle iteration after each run: it would stamp over the merge's rows)

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "pt-bpe_amd"))
import torch  # noqa: E402,F401
from geobpe import _native, synth  # noqa: E402
from geobpe.engine import GeoBPEEngine  # noqa: E402

iters = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "100,400,800").split(",")]
corpus = synth.make_corpus(synth.make_lengths(100_000, 40, 560, seed=0), seed=0)
eng = GeoBPEEngine(corpus, 5, tail=0).initialize()
eng.bin()
L = _native.lib()
F = {10: "F.start", 11: "F.setup", 15: "F.walked", 16: "F.deduped", 17: "F.resolved", 12: "F.rounds", 13: "F.end"}
A = {30: "A.start", 32: "A.counted", 33: "A.grown", 35: "A.end"}
done = 0
for it in iters:
    eng.run(it - done - 2)
    done = it - 2
    m = L.geobpe_debug_timeline(eng._ctx, 1, None, 0)
    eng.run(2)
    done += 2
    eng.synchronize()
    buf = np.zeros(m, dtype=np.int64)
    L.geobpe_debug_timeline(eng._ctx, 0, buf.ctypes.data_as(ctypes.c_void_p), m)
    t = buf.reshape(-1, 64)
    nwg = t.shape[0]
    G = 256 - 32 if nwg >= 256 else nwg - 32
    fr, ar = t[:G], t[G:G + 32]
    base = fr[:, 10][fr[:, 10] > 0].min()
    last = eng.merges[-1]
    print(f"merge {it}: count {last[1]} merged {last[2]}  find rows {G}, append rows 32")
    for rows, names in ((fr, F), (ar, A)):
        for k, nm in names.items():
            col = rows[:, k]
            col = col[col > 0]
            if len(col) == 0:
                continue
            rel = (col - base) / 100.0
            print(f"  {nm:12s} min {rel.min():8.1f}  med {np.median(rel):8.1f}  max {rel.max():8.1f}")
eng.close()
