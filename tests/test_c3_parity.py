"""The north_star target: bit-exact parity on the 10^5-sequence corpus.

BASELINE configs[2] (C3): 100 000 synthetic chains, lengths U{40..560} (~30 M
residues), seed 0, bins {1: 5}, 1000 merges -- the HIP loop (device-resident
``run()``) against the CPU oracle on the same corpus: merge list (key string and
count), segmentation and encoded ids.  configs[4] in its bins {1: 5} form (5000
merges on the same corpus) and configs[3] (the corpus row-sharded
over 8 ranks) are checked against the same oracle run.  Reference semantics:
foldingdiff/bpe.py:1431-1474 (bin), :1792-2166 (step), tokenizer.py:379-392 and
bpe.py:918-956 (encode)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

C3_MERGES = 1000
C5_MERGES = 5000


@pytest.fixture(scope="module")
def c3(oracle_lib):
    from geobpe import synth
    lengths = synth.make_lengths(100_000, 40, 560, seed=0)
    corpus = synth.make_corpus(lengths, seed=0)
    o = oracle_lib.OracleBPE(corpus, 5).initialize()
    o.bin()
    snap = {}
    for target in (C3_MERGES, C5_MERGES):
        while len(o.merges) < target:
            assert o.step() is not None
        snap[target] = dict(merges=list(o.merges), seg=o.segmentation(), enc=o.encode(),
                            thresholds=o.thresholds)
    del o
    return corpus, snap


def _check(run, want):
    assert run.merge_keys() == want["merges"]
    for x, y in zip(run.segmentation(), want["seg"]):
        assert np.array_equal(x, y)
    for x, y in zip(run.encode(), want["enc"]):
        assert np.array_equal(x, y)


@pytest.mark.timeout(600)
def test_c3_1000_merges_match_oracle(c3):
    from geobpe.engine import GeoBPEEngine
    corpus, snap = c3
    eng = GeoBPEEngine(corpus, 5, device=0).initialize()
    assert eng.thresholds == snap[C3_MERGES]["thresholds"]
    eng.bin()
    assert eng.run(C3_MERGES) == C3_MERGES
    _check(eng, snap[C3_MERGES])
    assert eng.verify_counts() == 0
    # configs[4] (bins {1: 5} form): the same loop on to 5000 merges
    assert eng.run(C5_MERGES - C3_MERGES) == C5_MERGES - C3_MERGES
    _check(eng, snap[C5_MERGES])
    assert eng.verify_counts() == 0
    eng.close()


@pytest.mark.timeout(900)
def test_c4_world8_matches_oracle(c3):
    """configs[3]: the C3 corpus row-sharded over 8 ranks (8 engines on one GPU,
    per-merge delta exchange), 1000 merges, bit-exact with the 1-rank oracle."""
    from geobpe.dist import VirtualCluster
    corpus, snap = c3
    vc = VirtualCluster(corpus, 5, world=8).initialize()
    assert vc.thresholds == snap[C3_MERGES]["thresholds"]
    vc.bin()
    for _ in range(C3_MERGES):
        assert vc.step() is not None
    _check(vc, snap[C3_MERGES])
    vc.close()
