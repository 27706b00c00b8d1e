"""Host-side logic that needs no GPU: the C-ABI library loads and exports every
symbol include/geobpe.h declares, the threshold edges and the row sharding."""
import os
import re

import numpy as np
import pytest

from conftest import REPO, load_golden


def _declared_symbols():
    src = open(os.path.join(REPO, "include", "geobpe.h")).read()
    return sorted(set(re.findall(r"\b(geobpe_[a-z_]+)\s*\(", src)))


def test_library_exports_header_symbols():
    from geobpe import _native, build
    build.build()
    L = _native.lib()  # loads libgeobpe.so (no compute calls without a GPU)
    declared = _declared_symbols()
    assert len(declared) >= 25
    for s in declared:
        assert hasattr(L, s), s
    assert sorted(_native.EXPORTED_SYMBOLS) == declared


def test_histogram_edges_match_numpy():
    from geobpe.engine import histogram_edges
    rng = np.random.default_rng(0)
    for B in (1, 2, 5, 12, 100):
        a = (rng.normal(-1, 2, 1000) + 2 * np.pi) % (2 * np.pi)
        _, e = np.histogram(a, bins=B)
        assert np.array_equal(histogram_edges(a.min(), a.max(), len(a), B), e)
    _, e = np.histogram(np.array([1.5, 1.5]), bins=3)  # degenerate range -> +-0.5
    assert np.array_equal(histogram_edges(1.5, 1.5, 2, 3), e)
    _, e = np.histogram(np.zeros(0), bins=4)
    assert np.array_equal(histogram_edges(np.inf, -np.inf, 0, 4), e)


def test_init_bond_angle_matches_reference_thresholds():
    """The tau histogram includes Tokenizer._init_bond_angle (bpe.py:845-846)."""
    from geobpe.engine import init_bond_angle
    import oracle.prologue as P
    assert init_bond_angle() == P.init_bond_angle()
    meta, corpus, _ = load_golden("g25x1-12_b3_short")
    thr = meta["thresholds"]["tau"]
    w = (init_bond_angle() + 2 * np.pi) % (2 * np.pi)
    assert thr[0][0] <= w <= thr[-1][1]


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_shard_rows_balanced_contiguous(world):
    from geobpe.dist import shard_rows, slice_corpus
    from geobpe import synth
    lengths = synth.make_lengths(97, 40, 560, seed=1)
    c = synth.make_corpus(lengths, seed=1)
    b = shard_rows(c["row_off"], world)
    assert b[0][0] == 0 and b[-1][1] == 97
    assert all(b[i][1] == b[i + 1][0] for i in range(world - 1))
    R = int(c["row_off"][-1])
    sizes = [int(c["row_off"][hi] - c["row_off"][lo]) for lo, hi in b]
    assert sum(sizes) == R
    assert max(sizes) - min(sizes) <= 2 * 560
    parts = [slice_corpus(c, lo, hi) for lo, hi in b]
    assert np.array_equal(np.concatenate([p["phi"] for p in parts]), c["phi"], equal_nan=True)
