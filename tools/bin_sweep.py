"""Time the dense bin pass (k_bin_count / k_bin_claim / k_bin_assign) on the C3
corpus for a few k_bin_count grid sizes (GEOBPE_BIN_GRID)."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "pt-bpe_amd"))
import torch  # noqa: E402

from geobpe import synth  # noqa: E402
from geobpe.engine import GeoBPEEngine  # noqa: E402

lengths = synth.make_lengths(100_000, 40, 560, seed=0)
corpus = synth.make_corpus(lengths, seed=0)
for arg in (sys.argv[1:] or ["256", "512", "1024"]):
    grid, _, mode = arg.partition(":")
    os.environ["GEOBPE_BIN_GRID"] = grid
    os.environ["GEOBPE_BIN_MODE"] = mode or "0"
    for rep in range(2):
        e = GeoBPEEngine(corpus, 5, device=0).initialize()
        e.set_profiling(True)
        e.bin()
        torch.cuda.synchronize()
        ms = {k: round(e.kernel_ms(k)[0] * 1000, 1) for k in ("bin_sample", "pair_count", "bin_claim", "bin_assign")}
        print(arg, rep, ms, "total_us", round(sum(ms.values()), 1), "keys", e.num_keys, flush=True)
        e.close()
