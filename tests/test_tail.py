"""The middle-regime and late-merge paths (csrc/mid.h k_mid_sel + k_mid_find, csrc/tail.h
k_tail): the same merges as the full-grid kernels and the CPU oracle, bit-exact (merge list
with key strings and counts, encoded ids, incremental counts = a full recount), whether
the switches happen at the first merge, mid-run or never.  Reference semantics:
foldingdiff/bpe.py:1792-2166 (step)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ALL_TAIL = 1 << 30  # every merge after the first runs in k_tail


def _corpus(n, lo, hi, seed, rep):
    from geobpe import synth
    return synth.make_corpus(synth.make_lengths(n, lo, hi, seed=seed), seed=seed, repeat_frac=rep)


def _oracle(oracle_lib, corpus, B, n):
    o = oracle_lib.OracleBPE(corpus, B).initialize()
    o.bin()
    for _ in range(n):
        if o.step() is None:
            break
    return o


# (mid, tail) thresholds: full-grid only, mid only, full-grid -> mid, mid -> tail,
# full-grid -> mid -> tail, tail only
REGIMES = [(0, 0), (ALL_TAIL, 0), (500, 0), (ALL_TAIL, 150), (600, 100), (0, ALL_TAIL)]


@pytest.mark.parametrize("mid, tail", REGIMES)
@pytest.mark.parametrize("cfg", [
    dict(n=2000, lo=40, hi=300, B=5, merges=400, seed=21, rep=0.0),
    dict(n=500, lo=40, hi=200, B=2, merges=400, seed=22, rep=0.05),  # long tokens, long runs
    dict(n=300, lo=1, hi=40, B=3, merges=300, seed=24, rep=0.2),     # 1-residue chains, repeats
    dict(n=800, lo=30, hi=250, B=12, merges=250, seed=23, rep=0.0),  # two-digit bins
])
def test_regimes_match_oracle(cfg, mid, tail, oracle_lib):
    from geobpe.engine import GeoBPEEngine
    corpus = _corpus(cfg["n"], cfg["lo"], cfg["hi"], cfg["seed"], cfg["rep"])
    o = _oracle(oracle_lib, corpus, cfg["B"], cfg["merges"])
    eng = GeoBPEEngine(corpus, cfg["B"], device=0, tail=tail, mid=mid).initialize()
    eng.bin()
    done = eng.run(10) + eng.run(cfg["merges"] - 10)
    assert done == len(o.merges)
    assert eng.merge_keys() == o.merges
    assert eng.verify_counts() == 0
    e, eo = eng.encode()
    oe, oo = o.encode()
    assert np.array_equal(e, oe) and np.array_equal(eo, oo)
    eng.close()


@pytest.mark.parametrize("mid, tail", [(0, ALL_TAIL), (ALL_TAIL, 0)])
def test_step_by_step_and_exhaustion(mid, tail, oracle_lib):
    """step() in the late-merge / middle-regime path, then run() to exhaustion (hot-list
    rebuilds and the end handled by k_commit / k_mid_find)."""
    from geobpe.engine import GeoBPEEngine
    corpus = _corpus(200, 5, 60, 31, 0.3)
    o = _oracle(oracle_lib, corpus, 3, 10 ** 6)
    eng = GeoBPEEngine(corpus, 3, device=0, tail=tail, mid=mid).initialize()
    eng.bin()
    for _ in range(40):
        assert eng.step() is not None
    eng.run(10 ** 6)
    assert eng.step() is None
    assert eng.merge_keys() == o.merges
    assert eng.verify_counts() == 0
    s, ids, off = eng.segmentation()
    os_, oids, ooff = o.segmentation()
    assert np.array_equal(s, os_) and np.array_equal(ids, oids) and np.array_equal(off, ooff)
    eng.close()


def test_merge_events_match_full_grid():
    """The merge-event log (the checkpoint's merge tree) of the middle-regime and late-merge
    paths equals the full-grid kernels'."""
    from geobpe.engine import GeoBPEEngine
    corpus = _corpus(400, 20, 120, 33, 0.1)
    out = []
    for mid, tail in ((0, 0), (0, ALL_TAIL), (ALL_TAIL, 0)):
        eng = GeoBPEEngine(corpus, 5, device=0, tail=tail, mid=mid).initialize()
        eng.record_events(True)
        eng.bin()
        eng.run(150)
        a, b, off = eng.events()
        out.append((eng.merge_keys(), a, b, off))
        eng.close()
    for o in out[1:]:
        assert out[0][0] == o[0]
        for x, y in zip(out[0][1:], o[1:]):
            assert np.array_equal(x, y)
