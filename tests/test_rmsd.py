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


def _kmed_both(D, k, seed, max_iterations=10):
    """the numpy loop of oracle/rmsd.py and the product's C step, from the same seed"""
    from geobpe import rmsd
    from oracle import rmsd as orm
    return [[int(x) for x in f(D, k, max_iterations, rng=np.random.default_rng(seed))]
            for f in (orm.k_medoids_from_matrix, rmsd.k_medoids_from_matrix)]


def test_k_medoids_c_step_equals_numpy_loop(ref):
    """csrc/rmsdkey.c kmed_step (numpy's float32 pairwise row sums and argmin rules in C)
    gives the numpy loop's medoids: the reference's matrices, random ones of every size the
    summation splits differently (below 8, up to 128, halves above), tied and quantised
    values, empty clusters (rng re-seeds) and a NaN."""
    for D, k, s in ((ref["D_ref"], 5, 3), (ref["D3_ref"], 4, 5)):
        a, b = _kmed_both(D, k, s)
        assert a == b
    g = np.random.default_rng(11)
    for n in (1, 2, 3, 7, 8, 9, 15, 16, 17, 100, 127, 128, 129, 136, 255, 256, 257, 300, 500):
        for trial in range(3):
            X = g.random((n, 3)) * 10
            D = np.sqrt(((X[:, None] - X[None]) ** 2).sum(-1)).astype(np.float32)
            if trial == 1:
                D = np.round(D * 2) / 2  # (ties everywhere)
            if trial == 2:
                D = g.random((n, n)).astype(np.float32) * 1e4  # (asymmetric, large sums)
            for k in (1, 2, 5, 9):
                a, b = _kmed_both(D, k, 100 * n + trial)
                assert a == b, (n, trial, k)
    for n in (9, 40, 128, 200, 333):  # (every row a permutation of one multiset: the medoid is
        #                                decided by the summation order's rounding alone)
        v = (g.random(n) * 1e3).astype(np.float32)
        D = np.stack([g.permutation(v) for _ in range(n)])
        a, b = _kmed_both(D, 1, n)
        assert a == b, n
        sums = D.sum(axis=1)
        assert len(set(sums.tolist())) > 1 or n < 16  # (the order does change the sums)
    D = np.zeros((12, 12), dtype=np.float32)  # (every row ties: all to medoid 0, the rest empty)
    a, b = _kmed_both(D, 4, 1)
    assert a == b
    D = g.random((40, 40)).astype(np.float32)
    D[5, 7] = np.nan
    a, b = _kmed_both(D, 3, 2)
    assert a == b


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
def test_device_scratch_release(ref):
    """geobpe_arena_release frees the per-device arenas; the next calls re-create them and
    give the same bits (arenas were kept for the process's lifetime)."""
    from geobpe import rmsd
    D1 = rmsd.rmsd_matrix(ref["A"])
    rmsd.release_scratch(0)
    D2 = rmsd.rmsd_matrix(ref["A"])
    rmsd.release_scratch()
    assert np.array_equal(D1, D2)


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


def _nerf_cases(ref):
    from geobpe.synth import COLUMNS
    ro = ref["nerf_row_off"]
    chains = [{c: ref[f"nerf_{c}"][ro[i]:ro[i + 1]] for c in COLUMNS} for i in range(len(ro) - 1)]
    want = [ref["nerf_coords"][a:b] for a, b in zip(ref["nerf_coff"][:-1], ref["nerf_coff"][1:])]
    return chains, ref["nerf_spans"], want


def test_oracle_nerf_matches_reference(ref):
    """The numpy NeRF restatement on token_geo spans equals the reference's
    Tokenizer.compute_coords (tokenizer.py:347-363) to 1e-9."""
    from geobpe.rmsd import token_geo
    from oracle import rmsd as orm
    chains, spans, want = _nerf_cases(ref)
    for (ci, index, length), w in zip(spans, want):
        cols = chains[ci]
        n = len(cols["phi"])
        length = min(int(length), 3 * n - 1 - int(index))
        start = 3 * (int(index) // 3)
        end = 3 * (((int(index) + length - 1) + 1) // 3) + 1
        c = orm.nerf(token_geo(cols, start, end - start + 1))
        c = c[int(index) - start: len(c) - (end - (int(index) + length - 1))]
        assert c.shape == w.shape and np.max(np.abs(c - w)) <= TOL64


@pytest.mark.gpu
def test_device_nerf_matches_reference(ref):
    """geobpe.rmsd.compute_coords (device k_nerf) equals the reference's
    Tokenizer.compute_coords for whole chains, single residues, the 2-bond last
    residue and spans that start or end inside a residue."""
    from geobpe import rmsd
    chains, spans, want = _nerf_cases(ref)
    for ci in range(len(chains)):
        sel = [k for k in range(len(spans)) if spans[k][0] == ci]
        got = rmsd.compute_coords(chains[ci], [(int(spans[k][1]), int(spans[k][2])) for k in sel])
        for k, g in zip(sel, got):
            assert g.shape == want[k].shape and np.max(np.abs(g - want[k])) <= TOL64


@pytest.mark.gpu
def test_device_nerf_featurize_round_trip():
    """NeRF then featurisation (csrc/featurize.h) recovers the internal coordinates:
    the device's two geometry directions are inverse to each other on 2000 chains."""
    from geobpe import pdb, rmsd, synth
    corpus = synth.make_corpus(synth.make_lengths(2000, 5, 80, seed=13), seed=13)
    ro = corpus["row_off"]
    geos = []
    for i in range(len(ro) - 1):
        cols = {c: corpus[c][ro[i]:ro[i + 1]] for c in synth.COLUMNS}
        n = ro[i + 1] - ro[i]
        g = rmsd.token_geo(cols, 0, 3 * n - 1)
        g["N:CA"] = [1.46] * n  # featurisation measures the placed bonds; init bonds are the first residue's
        g["CA:C"] = [1.54] * n
        geos.append(g)
    xyz = rmsd.geo_coords(geos)
    feat = pdb.featurize([x.reshape(-1, 3, 3) for x in xyz])
    for i in range(0, len(ro) - 1, 97):
        a, b = ro[i], ro[i + 1]
        for c in ("phi", "psi", "omega", "CA:C:1N", "C:1N:1CA"):
            v, w = feat[c][feat["row_off"][i]:feat["row_off"][i + 1]], corpus[c][a:b]
            m = ~np.isnan(w)
            d = np.angle(np.exp(1j * (v[m] - w[m])))
            assert np.max(np.abs(d)) < 1e-9, c
