"""Time the k-medoids distance matrix (max_num_strucs = 500 structures) on the
device against the numpy restatement of compute_rmsd (one core)."""
import os
import sys
import time

import numpy as np

here = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(here, "..", "..", "pt-bpe_amd"))
sys.path.insert(0, os.path.join(here, "..", ".."))
from geobpe import rmsd  # noqa: E402
from oracle import rmsd as orm  # noqa: E402

rng = np.random.default_rng(7)
for atoms in (4, 31, 91):
    S = np.cumsum(rng.normal(size=(500, atoms, 3)), axis=1)
    rmsd.rmsd_matrix(S)
    t = time.perf_counter()
    for _ in range(5):
        rmsd.rmsd_matrix(S)
    tg = (time.perf_counter() - t) / 5
    t = time.perf_counter()
    n = 0
    for i in range(0, 500, 25):
        for j in range(i, 500):
            orm.rmsd(S[i], S[j])
            n += 1
    tc = (time.perf_counter() - t) / n * 500 * 501 / 2
    print(f"atoms {atoms}: device {tg * 1e3:.2f} ms (host round trip incl.), numpy 1 core {tc:.2f} s (extrapolated)")
