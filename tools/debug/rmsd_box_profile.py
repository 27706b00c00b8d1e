"""cProfile of bench.py --config rmsd's timed steps on the GPU box (the README downstream setting,
2 000 synthetic chains): the top functions by own and cumulative time, to stderr.

  python tools/debug/rmsd_box_profile.py [chains] [steps]"""
import cProfile
import io
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "pt-bpe_amd"))

import torch  # noqa: E402,F401  (the HIP runtime shared with torch)
from geobpe import synth  # noqa: E402
from geobpe.bpe import BPE  # noqa: E402

argv = [a for a in sys.argv[1:] if not a.startswith("--")]
n = int(argv[0]) if len(argv) > 0 else 2000
steps = int(argv[1]) if len(argv) > 1 else 60
corpus = synth.make_corpus(synth.make_lengths(n, 40, 560, seed=0), seed=0)
bpe = BPE(corpus, bins={1: 50}, bin_strategy="histogram", res_init=True, std_bonds=False,
          rmsd_partition_min_size=0, rmsd_super_res=True, num_partitions={2: 2, 3: 5, 5: 1, 6: 2, 8: 1},
          max_num_strucs=500, glue_opt=True, glue_opt_prior=0.0, glue_opt_every=10, glue_opt_method="all",
          seed=0, device=0)
bpe.initialize()
bpe.glue_opt_all()
bpe.bin()
bpe.run(5)
pr = cProfile.Profile()
t0 = time.perf_counter()
pr.enable()
bpe.run(steps)
pr.disable()
T = time.perf_counter() - t0
print(f"{steps} steps: {1000 * T / steps:.2f} ms a step (under cProfile)", file=sys.stderr)
for key in ("tottime", "cumulative"):
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats(key).print_stats(30)
    print(s.getvalue(), file=sys.stderr)
