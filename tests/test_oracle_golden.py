"""The CPU oracle against the reference's own outputs (tests/golden, made by
tests/golden/make_golden.py from /root/reference foldingdiff/bpe.py)."""
import json

import numpy as np
import pytest

from conftest import golden_names, load_golden


@pytest.mark.parametrize("name", golden_names())
def test_oracle_matches_reference(name, oracle_lib):
    meta, corpus, arrs = load_golden(name)
    B = meta["bins"]["1"]
    cover = meta.get("bin_strategy", "histogram") == "histogram-cover"
    o = oracle_lib.OracleBPE(corpus, B, cover=cover, strategy=meta.get("bin_strategy")).initialize()
    # thresholds (bpe.py:820-876) and first-appearance labels (bpe.py:231-261)
    assert o.thresholds == {k: [tuple(p) for p in v] for k, v in meta["thresholds"].items()}
    assert np.array_equal(o.labels, arrs["init_labels"])
    assert o.K0 == meta["K0"]
    o.bin()
    for _ in range(len(meta["merges"])):
        assert o.step() is not None
    # merge list: key string + count per iteration
    assert [list(m) for m in o.merges] == meta["merges"]
    s, ids, off = o.segmentation()
    assert np.array_equal(s, arrs["seg_start"]) and np.array_equal(ids, arrs["seg_id"])
    assert np.array_equal(off, arrs["seg_off"])
    e, eoff = o.encode()
    assert np.array_equal(e, arrs["ids"]) and np.array_equal(eoff, arrs["ids_off"])
    assert {str(k): v for k, v in o.vocab().items()} == meta["vocab"]
    assert o.vocab_size == meta["vocab_size"]


def test_oracle_get_ind_semantics(oracle_lib):
    from oracle.prologue import get_ind, get_ind_vec
    thr = [(0.0, 1.0), (1.0, 2.0), (2.0, 3.0)]
    assert get_ind(0.0, thr) == 0 and get_ind(1.0, thr) == 1 and get_ind(3.0, thr) == 2
    for bad in (-0.1, 3.0000001, float("nan")):
        with pytest.raises(ValueError):
            get_ind(bad, thr)
        with pytest.raises(ValueError):
            get_ind_vec(np.array([bad]), thr)
    v = np.array([0.0, 0.5, 1.0, 2.999, 3.0])
    assert get_ind_vec(v, thr).tolist() == [get_ind(x, thr) for x in v]


def test_oracle_out_of_range_raises(oracle_lib):
    """A value the histogram excluded (exact 0.0, bpe.py:844) but a key uses -> ValueError."""
    meta, corpus, _ = load_golden("g40x50_b5")
    corpus = {k: v.copy() for k, v in corpus.items()}
    corpus["psi"][3] = 0.0  # wrap(0)=0 < every other wrapped psi
    o = oracle_lib.OracleBPE(corpus, 5)
    with pytest.raises(ValueError):
        o.initialize()
