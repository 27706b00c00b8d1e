"""A/B of the regime thresholds on the C3 corpus: merges 11..N timed for each mid:tail
pair (0 = never); per-kernel event times (a second, event-timed run) and the counts.
usage: python tools/tail_ab.py N mid:tail [mid:tail ...]"""
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
    pairs = [tuple(int(v) for v in x.split(":")) for x in sys.argv[2:]]
    corpus = synth.make_corpus(synth.make_lengths(100_000, 40, 560, seed=0), seed=0)
    for mid, tail in pairs:
        e = GeoBPEEngine(corpus, 5, device=0, tail=tail, mid=mid, max_vocab=1 << 20).initialize()
        e.bin()
        e.run(10)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        done = e.run(n - 10)
        T = time.perf_counter() - t0
        m = e.merges
        e.close()
        e = GeoBPEEngine(corpus, 5, device=0, tail=tail, mid=mid, max_vocab=1 << 20).initialize()
        e.bin()
        e.run(10)
        e.set_profiling(True, only="select,find,commit,tail,tail_build,place")
        e.set_work_counters(False)
        e.set_hold(3000)
        e.run(n - 10)
        ks = {k: e.kernel_ms(k) for k in ("select", "find", "commit", "tail", "tail_build", "place")}
        assert e.merges == m
        # counts around the switch
        out = {"mid": mid, "tail": tail, "merges": done, "ms": round(T * 1000, 2), "merges_per_s": round(done / T, 1),
               "kernels_ms": {k: [round(v[0], 3), v[1]] for k, v in ks.items()},
               "counts": [m[i][1] for i in (10, 50, 100, 200, 300, 400, 500, 700, 900, len(m) - 1) if i < len(m)]}
        print(json.dumps(out), flush=True)
        e.close()


if __name__ == "__main__":
    main()
