"""Host-side profile of the RMSD-partitioned mode's step() (RmsdBPE) on the CPU: the device
batches (NeRF, Kabsch RMSD, thresholds) replaced by the oracle's numpy restatements, as in
tests/test_rmsd_mode.py's host path, so that what is left is the host bookkeeping the GPU box
also runs.  Prints the mean step time less the stand-ins' own time, and the top functions.

  python tools/debug/rmsd_host_profile.py [N LO HI STEPS]   (default 2000 40 120 50)"""
import cProfile
import os
import pstats
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "pt-bpe_amd"))
sys.path.insert(0, ROOT)

import oracle.prologue as prologue  # noqa: E402
import oracle.rmsd as orm  # noqa: E402
from geobpe import rmsd, rmsd_bpe, synth  # noqa: E402
from geobpe.bpe import BPE  # noqa: E402

n, lo, hi, steps = (int(x) for x in (sys.argv[1:5] if len(sys.argv) >= 5 else (2000, 40, 120, 50)))
stand = [0.0]


def timed(f):
    def g(*a, **k):
        t0 = time.perf_counter()
        r = f(*a, **k)
        stand[0] += time.perf_counter() - t0
        return r
    return g


rmsd.geo_coords = timed(lambda geos, device=0: [orm.nerf(g) for g in geos])
rmsd.nerf_packed = timed(lambda off, packed, device=0: orm.nerf_packed(off, packed))
rmsd.nerf_atoms = timed(lambda off, packed, device=0: orm.nerf_atoms(off, packed))
rmsd.rmsd_matrix = timed(lambda S, device=0: orm.rmsd_matrix(S))
rmsd.rmsd_cross = timed(lambda A, B, device=0: np.array([[orm.rmsd(a, b) for b in B] for a in A]))
rmsd_bpe.RmsdBPE._grid_thresholds = lambda self: {s: prologue.thresholds(self._corpus, b) for s, b in self.bins.items()}

corpus = synth.make_corpus(synth.make_lengths(n, lo, hi, seed=31), seed=31)
bpe = BPE(corpus, bins={1: 5}, res_init=True, rmsd_partition_min_size=0, rmsd_super_res=True,
          num_partitions={2: 2, 3: 5, 5: 2, 8: 1}, max_num_strucs=500, seed=0)
bpe.initialize()
bpe.bin()
bpe.run(5)  # (warm)
s0 = stand[0]
prof = cProfile.Profile()
t0 = time.perf_counter()
prof.enable()
done = bpe.run(steps)
prof.disable()
t = time.perf_counter() - t0
print(f"{done} steps: {1000 * t / done:.2f} ms per step, of which stand-ins {1000 * (stand[0] - s0) / done:.2f} ms; "
      f"host {1000 * (t - (stand[0] - s0)) / done:.2f} ms per step")
pstats.Stats(prof).sort_stats("tottime").print_stats(18)
