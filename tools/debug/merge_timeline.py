"""Phase timeline of k_find / k_commit (and k_select) for a few merges on the C3
corpus (geobpe_debug_timeline): per-workgroup wall-clock stamps (100 MHz), relative
to the first k_commit start."""
import ctypes
import os
import sys

os.environ.setdefault("GEOBPE_SPEC", "0")  # (no idle iteration after each run: it would stamp over the merge's rows)

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "pt-bpe_amd"))
import torch  # noqa: E402,F401
from geobpe import _native, synth  # noqa: E402
from geobpe.engine import GeoBPEEngine  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
iters = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "1,6,20,200,800").split(",")]
corpus = synth.make_corpus(synth.make_lengths(n, 40, 560, seed=0), seed=0)
eng = GeoBPEEngine(corpus, 5).initialize()
eng.bin()
L = _native.lib()
names = {0: "C.start", 1: "C.init", 2: "C.records", 3: "C.resolved", 4: "C.published", 5: "C.flush+klist", 6: "C.end",
         10: "F.start", 11: "F.setup", 14: "F.r0.queued", 15: "F.r0.walked", 16: "F.r0.grouped", 12: "F.walked",
         13: "F.end", 40: "F.w.T1", 41: "F.w.T2", 42: "F.w.T3", 43: "F.w.emitted", 44: "F.w.hashed", 30: "P.start", 38: "P.scanned", 37: "P.issued", 31: "P.tokens", 32: "P.slots", 33: "P.end",
         50: "C.i.loaded", 51: "C.i.zeroed", 53: "C.published0", 56: "C.r.first", 57: "C.r.extras", 58: "C.r.decs", 20: "S.start", 21: "S.scanned", 22: "S.max", 23: "S.ties", 24: "S.staged", 25: "S.tourn", 26: "S.end"}
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
        print(f"merge {it}: (no stamps)")
        continue
    vals = {7: "C.records(n)", 8: "C.decrements(n)", 9: "C.keys(n)", 54: "C.extras(n)", 55: "C.overflow(n)",
            59: "C.dec_extras(n)", 60: "F.scanned(n+1)", 61: "F.cands(n+1)", 62: "F.occs(n+1)"}
    vv = t[:, [7, 8, 9, 54, 55, 59]].copy()
    fv = t[:, [60, 61, 62]].copy() - 1
    for k, nm in vals.items():  # values, not times
        v = t[:, k][t[:, k] > 0]
        if len(v):
            print(f"  {nm:14s} min {v.min():8d}  med {int(np.median(v)):8d}  max {v.max():8d}  sum {v.sum()}")
        t[:, k] = 0
    base = t[:, 0][t[:, 0] > 0].min() if (t[:, 0] > 0).any() else t[t > 0].min()
    rel = (t - base) / 100.0
    rel[t == 0] = np.nan
    last = eng.merges[-1]
    print(f"merge {it}: count {last[1]} merged {last[2]}  workgroups {len(t)}")
    cols = [k for k in range(64) if not np.all(np.isnan(rel[:, k]))]
    for k in sorted(cols, key=lambda k: np.nanmedian(rel[:, k])):
        col = rel[:, k]
        print(f"  {names.get(k, str(k)):14s} min {np.nanmin(col):8.1f}  med {np.nanmedian(col):8.1f}  max {np.nanmax(col):8.1f}")
    if not np.all(np.isnan(rel[:, 6])):  # the slowest commit workgroups and their work
        order = np.argsort(-np.nan_to_num(rel[:, 6], nan=-1e9))[:6]
        print("  slowest commit workgroups: wg  init  r.first r.extras r.decs records  resolved  pub0  published  end"
              " | krec  drec  keys  extras  ovf  dec_extras")
        for w in order:
            print(f"    {w:4d} " + " ".join(f"{rel[w, k]:7.1f}" for k in (1, 56, 57, 58, 2, 3, 53, 4, 6))
                  + f" | {vv[w, 0]:5d} {vv[w, 1]:5d} {vv[w, 2]:5d} {vv[w, 3]:5d} {vv[w, 4]:5d} {vv[w, 5]:5d}")
        print(f"  median work: krec {int(np.median(vv[:, 0]))} drec {int(np.median(vv[:, 1]))} keys {int(np.median(vv[:, 2]))}")
    if not np.all(np.isnan(rel[:, 13])):  # the slowest find workgroups and their work
        order = np.argsort(-np.nan_to_num(rel[:, 13], nan=-1e9))[:6]
        print("  slowest find workgroups: wg  start  setup  queued  T1  r0.walked  grouped  walked  end | scanned  cands  occs")
        for w in order:
            print(f"    {w:4d} " + " ".join(f"{rel[w, k]:7.1f}" for k in (10, 11, 14, 40, 15, 16, 12, 13))
                  + f" | {fv[w, 0]:6d} {fv[w, 1]:6d} {fv[w, 2]:6d}")
        print(f"  median find work: scanned {int(np.median(fv[:, 0]))} cands {int(np.median(fv[:, 1]))} "
              f"occs {int(np.median(fv[:, 2]))}")
eng.close()
