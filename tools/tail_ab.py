"""A/B of the late-merge threshold on the C3 corpus: merges 11..N timed for each
`tail` value (0 = full-grid kernels only); per-kernel event times and the merge at
which the switch happened.  usage: python tools/tail_ab.py N tail [tail ...]"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "pt-bpe_amd"))


def main():
    import torch
    from geobpe import synth
    from geobpe.engine import GeoBPEEngine
    n = int(sys.argv[1])
    tails = [int(x) for x in sys.argv[2:]]
    corpus = synth.make_corpus(synth.make_lengths(100_000, 40, 560, seed=0), seed=0)
    for tail in tails:
        e = GeoBPEEngine(corpus, 5, device=0, tail=tail, max_vocab=1 << 20).initialize()
        e.bin()
        e.run(10)
        e.set_profiling(True, only="select,find,commit,tail,tail_build")
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        done = e.run(n - 10)
        T = time.perf_counter() - t0
        ks = {k: e.kernel_ms(k) for k in ("select", "find", "commit", "tail", "tail_build")}
        m = e.merges
        # counts around the switch
        out = {"tail": tail, "merges": done, "ms": round(T * 1000, 2), "merges_per_s": round(done / T, 1),
               "kernels_ms": {k: [round(v[0], 3), v[1]] for k, v in ks.items()},
               "counts": [m[i][1] for i in (10, 50, 100, 200, 300, 400, 500, 700, 900, len(m) - 1) if i < len(m)]}
        print(json.dumps(out), flush=True)
        e.close()


if __name__ == "__main__":
    main()
