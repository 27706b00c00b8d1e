"""k_apply phase timeline in delta (multi-rank) mode at world size 1: the engine
exports / imports its own deltas through device buffers (no collective)."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "pt-bpe_amd"))
import torch  # noqa: E402
from geobpe import _native, synth  # noqa: E402
from geobpe.engine import GeoBPEEngine  # noqa: E402


class LocalGroup:
    world_size = 1
    force = True
    residue_base = 0

    def __init__(self, R):
        self.total_residues = R
        self.buf = torch.empty((3 * R + 65536) * 40, dtype=torch.uint8, device="cuda")
        self.cnt = torch.zeros(1, dtype=torch.int64, device="cuda")

    def reduce_ranges(self, mm, cnt, n):
        return mm, cnt, n

    def reduce_first(self, f):
        return f

    def export_buffer(self, e):
        return len(self.buf) // 40, ctypes.c_void_p(self.buf.data_ptr())

    def all_gather_deltas(self, e, n):
        e.synchronize()
        return ctypes.c_void_p(self.buf.data_ptr()), n

    def exchange_async(self, e):
        L = e.L
        e._chk(L.geobpe_delta_export_async(e._ctx, ctypes.c_void_p(self.buf.data_ptr()), len(self.buf) // 40,
                                           ctypes.c_void_p(self.cnt.data_ptr())))
        e.synchronize()
        n = int(self.cnt.item())
        e._chk(L.geobpe_delta_import_async(e._ctx, ctypes.c_void_p(self.buf.data_ptr()), n))


n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
iters = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "20,200").split(",")]
corpus = synth.make_corpus(synth.make_lengths(n, 40, 560, seed=0), seed=0)
g = LocalGroup(int(corpus["row_off"][-1]))
eng = GeoBPEEngine(corpus, 5, group=g).initialize()
eng.bin()
L = _native.lib()
done = 0
for it in iters:
    while done < it - 1:
        eng.step(want_merged=False)
        done += 1
    m = L.geobpe_debug_timeline(eng._ctx, 1, None, 0)
    eng.step(want_merged=False)
    done += 1
    buf = np.zeros(m, dtype=np.int64)
    L.geobpe_debug_timeline(eng._ctx, 0, buf.ctypes.data_as(ctypes.c_void_p), m)
    t = buf.reshape(-1, 64)
    t = t[t[:, 0] > 0]
    base = t[:, 0].min()
    rel = (t - base) / 100.0
    rel[t == 0] = np.nan
    print(f"merge {it}: workgroups {len(t)}")
    for k in range(64):
        col = rel[:, k]
        if np.all(np.isnan(col)):
            continue
        print(f"  stamp {k:2d} min {np.nanmin(col):8.1f}  med {np.nanmedian(col):8.1f}  max {np.nanmax(col):8.1f}")
