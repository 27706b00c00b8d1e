"""Structure side of the object API against the reference (tests/golden/recover_ref.*, made by
tests/golden/make_recover_golden.py): Tokenizer.compute_coords (tokenizer.py:347-363, the
current and the original geometry) and BPE.recover_structure(recover(dequantize(quantize(t))))
(bpe.py:986-1051, bin/train.py:715-716), for a scoped-mode run and an RMSD-mode run.

Recovered columns and bond_to_token are compared exactly; coordinates (NeRF, float64, on the
device here) within 1e-9 A.
"""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN

COLS = ["0C:1N", "N:CA", "CA:C", "phi", "psi", "omega", "tau", "CA:C:1N", "C:1N:1CA"]
TOL = 1e-9


def _ref():
    with open(os.path.join(GOLDEN, "recover_ref.json")) as f:
        meta = json.load(f)
    with np.load(os.path.join(GOLDEN, "recover_ref.npz"), allow_pickle=False) as z:
        arrs = {k: z[k] for k in z.files}
    return meta, arrs


def _load_fixture(name):
    with open(os.path.join(GOLDEN, name + ".json")) as f:
        m = json.load(f)
    with np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False) as z:
        corpus = {k: z[k] for k in COLS + ["row_off"]}
    return m, corpus


def _trained(case, meta):
    from geobpe.bpe import BPE
    fx, calls = meta[case]["fixture"], meta[case]["calls"]
    m, corpus = _load_fixture(fx)
    bins = {int(a): b for a, b in m["bins"].items()}
    if case == "scoped":
        bpe = BPE(corpus, bins=bins, res_init=True, rmsd_partition_min_size=float("inf"), seed=0)
        bpe.initialize()
        bpe.bin()
        assert bpe.run(calls) == calls
    else:
        bpe = BPE(corpus, bins=bins, rmsd_partition_min_size=m["rmsd_partition_min_size"],
                  rmsd_super_res=m["rmsd_super_res"], num_partitions={int(a): b for a, b in m["num_partitions"].items()},
                  max_num_strucs=m["max_num_strucs"], res_init=True, std_bonds=True, seed=0)
        bpe.initialize()
        bpe.bin()
        for _ in range(calls):
            bpe.step()
    return bpe


def check(case):
    meta, arrs = _ref()
    bpe = _trained(case, meta)
    for i in range(3):
        t = bpe.tokenizers[i]
        np.testing.assert_allclose(t.compute_coords(), arrs[f"{case}{i}_coords"], atol=TOL, rtol=0)
        np.testing.assert_allclose(t.compute_coords(orig=True), arrs[f"{case}{i}_coords_orig"], atol=TOL, rtol=0)
        dq = bpe.dequantize(bpe.quantize(t))
        t2 = bpe.recover_structure(bpe.recover(dq), dq)
        got = [[s0, list(v[1]) if isinstance(v[1], tuple) else v[1], v[2]] for s0, v in t2.bond_to_token.items()]
        assert got == meta[case]["btt"][i]
        for c in COLS:
            assert np.array_equal(np.asarray(t2._c.cur[c]), arrs[f"{case}{i}_rec_{c}"], equal_nan=True), c
        np.testing.assert_allclose(t2.compute_coords(), arrs[f"{case}{i}_rec_coords"], atol=TOL, rtol=0)
    assert sorted(bpe.init_structure(4)["angles"].columns) == sorted(COLS)


def test_rmsd_mode_recover_host(monkeypatch):
    """The RMSD mode's host logic with the oracle's numpy NeRF / Kabsch in place of the
    device batches (test infrastructure)."""
    import oracle.prologue as prologue
    import oracle.rmsd as orm
    from geobpe import rmsd, rmsd_bpe
    monkeypatch.setattr(rmsd, "geo_coords", lambda geos, device=0: [orm.nerf(g) for g in geos])
    monkeypatch.setattr(rmsd, "nerf_packed", lambda off, packed, device=0: orm.nerf_packed(off, packed))
    monkeypatch.setattr(rmsd, "nerf_atoms", lambda off, packed, device=0: orm.nerf_atoms(off, packed))
    monkeypatch.setattr(rmsd, "rmsd_matrix", lambda S, device=0: orm.rmsd_matrix(S))
    monkeypatch.setattr(rmsd, "rmsd_cross", lambda A, B, device=0: np.array([[orm.rmsd(a, b) for b in B] for a in A]))
    monkeypatch.setattr(rmsd_bpe.RmsdBPE, "_grid_thresholds",
                        lambda self: {s: prologue.thresholds(self._corpus, b) for s, b in self.bins.items()})
    check("rmsd")


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["scoped", "rmsd"])
def test_recover_and_coords_match_reference(case):
    check(case)
