"""RMSD partitioning primitives: the device Kabsch RMSD
(csrc/rmsd.h via geobpe.rmsd) and the k-medoids loop, against the reference's own
outputs (tests/golden/rmsd_ref.npz from foldingdiff/algo.py) and the numpy
restatement (oracle/rmsd.py).  Floating point: the distance matrix is float32 in
the reference, so the device matrix must agree to 2e-6 absolute (float32 rounding
of values up to ~10 A); the float64 cross matrix to 1e-9."""
import os

import numpy as np
import pytest

from conftest import GOLDEN

TOL32, TOL64 = 2e-6, 1e-9


@pytest.fixture(scope="module")
def ref():
    return dict(np.load(os.path.join(GOLDEN, "rmsd_ref.npz")))


def test_oracle_matches_reference_matrix(ref):
    from oracle import rmsd as orm
    assert np.max(np.abs(orm.rmsd_matrix(ref["A"]) - ref["D_ref"])) <= TOL32
    assert np.max(np.abs(orm.rmsd_matrix(ref["A3"]) - ref["D3_ref"])) <= TOL32
    cross = np.array([[orm.rmsd(a, b) for b in ref["B"]] for a in ref["A"]])
    assert np.max(np.abs(cross - ref["cross_ref"])) <= TOL64


def test_k_medoids_loop_matches_reference(ref):
    """The host iterations on the reference's own matrix: same rng draws, same medoids."""
    from geobpe.rmsd import k_medoids_from_matrix
    m = k_medoids_from_matrix(ref["D_ref"], 5, rng=np.random.default_rng(3))
    assert [int(x) for x in m] == ref["medoids_ref"].tolist()
    m3 = k_medoids_from_matrix(ref["D3_ref"], 4, rng=np.random.default_rng(5))
    assert [int(x) for x in m3] == ref["medoids3_ref"].tolist()


@pytest.mark.gpu
def test_device_rmsd_matches_reference(ref):
    from geobpe import rmsd
    D = rmsd.rmsd_matrix(ref["A"])
    assert D.dtype == np.float32 and np.max(np.abs(D - ref["D_ref"])) <= TOL32
    assert np.max(np.abs(rmsd.rmsd_matrix(ref["A3"]) - ref["D3_ref"])) <= TOL32
    assert np.max(np.abs(rmsd.rmsd_cross(ref["A"], ref["B"]) - ref["cross_ref"])) <= TOL64
    # rigid copies: ~0; mirror images: clearly not
    assert D[0, 1] < 1e-6 and D[12, 13] > 0.1


@pytest.mark.gpu
def test_device_k_medoids_and_assignment_match_reference(ref):
    from geobpe import rmsd
    m = rmsd.k_medoids(list(ref["A"]), 5, rng=np.random.default_rng(3))
    assert [int(x) for x in m] == ref["medoids_ref"].tolist()
    m3 = rmsd.k_medoids(list(ref["A3"]), 4, rng=np.random.default_rng(5))
    assert [int(x) for x in m3] == ref["medoids3_ref"].tolist()
    a = rmsd.assign(ref["A"], ref["B"])
    assert np.array_equal(a, np.argmin(ref["cross_ref"], axis=1))


@pytest.mark.gpu
def test_device_rmsd_at_max_num_strucs():
    """max_num_strucs = 500 structures of 31 atoms (a 10-residue token): the device
    matrix against the numpy restatement on sampled pairs, plus size-independent
    properties (zero diagonal, symmetry, invariance under a rigid motion)."""
    from geobpe import rmsd
    from oracle import rmsd as orm
    rng = np.random.default_rng(7)
    S = np.cumsum(rng.normal(size=(500, 31, 3)), axis=1)
    D = rmsd.rmsd_matrix(S)
    assert np.all(np.diag(D) < 1e-6) and np.array_equal(D, D.T)
    for i, j in rng.integers(0, 500, size=(200, 2)):
        assert abs(float(D[i, j]) - orm.rmsd(S[i], S[j])) <= TOL32 * max(1.0, orm.rmsd(S[i], S[j]))
    th = 0.7
    Rz = np.array([[np.cos(th), -np.sin(th), 0], [np.sin(th), np.cos(th), 0], [0, 0, 1]])
    X = rmsd.rmsd_cross(S[:20], S[:20] @ Rz.T + 3.0)
    assert np.all(np.abs(np.diag(X)) < 1e-9)
    assert np.max(np.abs(X - D[:20, :20].astype(np.float64))) <= TOL32 * 10
