"""RMSD partitioning primitives on the GPU (first part).

The reference's RMSD mode (``rmsd_partition_min_size`` < inf) clusters the
occurrences of a token with k-medoids under Kabsch RMSD and assigns every
occurrence to its nearest medoid:

  reference                                   here
  algo.compute_rmsd(P, Q)  algo.py:48-65      rmsd_cross([P], [Q])[0, 0]
  k_medoids' distance matrix algo.py:179-189  rmsd_matrix(strucs)   (float32, as there)
  algo.k_medoids(strucs, k, ..., rng)         k_medoids(...)        (same rng draws)
  nearest medoid per occurrence               assign(coords, medoids)
    bpe.py:645-657, 1764-1777

The distances come from ``geobpe_rmsd`` (csrc/rmsd.h: one thread per pair,
float64, Jacobi SVD of the 3x3 covariance, explicit residuals); the k-medoids
iterations are the reference's host loop, fed the device matrix.  The BPE step
itself still rejects RMSD partitioning (geobpe.bpe._check_scope): the medoid
geometry write-back and glue optimisation (LBFGS over NeRF) are not built.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _native


def _coords(strucs) -> np.ndarray:
    a = np.ascontiguousarray(np.asarray(strucs, dtype=np.float64))
    if a.ndim != 3 or a.shape[2] != 3:
        raise ValueError(f"structures must be (n, atoms, 3), got {a.shape}")
    return a


def _run(a: np.ndarray, b, symmetric: bool, device: int) -> np.ndarray:
    L = _native.lib()
    na, nat = a.shape[0], a.shape[1]
    nb = na if symmetric else b.shape[0]
    if not symmetric and b.shape[1] != nat:
        raise ValueError(f"atom counts differ: {nat} vs {b.shape[1]}")
    out = np.empty((na, nb), dtype=np.float64)
    if na * nb == 0:
        return out
    pb = None if symmetric else b.ctypes.data_as(ctypes.c_void_p)
    rc = L.geobpe_rmsd(int(device), na, nb, nat, a.ctypes.data_as(ctypes.c_void_p), pb, 1 if symmetric else 0,
                       out.ctypes.data_as(ctypes.c_void_p))
    if rc:
        raise _native.GeoBPEError(f"geobpe_rmsd failed (code {rc})")
    return out


def rmsd_cross(A, B, device: int = 0) -> np.ndarray:
    """float64 (len(A), len(B)): compute_rmsd(A_i, B_j) (B_j aligned onto A_i)."""
    return _run(_coords(A), _coords(B), False, device)


def rmsd_matrix(strucs, device: int = 0) -> np.ndarray:
    """k_medoids' distance matrix: float32 (N, N), upper triangle computed as
    compute_rmsd(strucs[i], strucs[j]) for j >= i and mirrored (algo.py:179-189)."""
    return _run(_coords(strucs), None, True, device).astype(np.float32)


def k_medoids(strucs, k, max_iterations: int = 10, tol: float = 1e-4, *, rng=None, device: int = 0):
    """algo.k_medoids (algo.py:144-213) on the device distance matrix: the same
    initial draw, assignment, medoid update, empty-cluster re-seed and stopping rule,
    with the same numpy Generator calls (so a seeded rng gives the same medoids)."""
    N = len(strucs)
    if min(N, k) == N:
        print(f"k-medoids: k=N={N}, every struc is a medoid")
        return list(range(N))
    return k_medoids_from_matrix(rmsd_matrix(strucs, device=device), k, max_iterations, tol, rng=rng)


def k_medoids_from_matrix(D: np.ndarray, k, max_iterations: int = 10, tol: float = 1e-4, *, rng=None):
    """The iterations of algo.k_medoids (algo.py:191-213) on a given distance matrix."""
    N = len(D)
    k = min(N, k)
    if rng is None:
        rng = np.random.default_rng(None)
    medoid_indices = rng.choice(np.arange(N), size=k, replace=False)
    assignments = np.zeros(N, dtype=int)
    for iteration in range(max_iterations):
        for i in range(N):
            assignments[i] = np.argmin(D[i, medoid_indices])
        total_shift = 0.0
        new_medoid_indices = []
        for j in range(k):
            members = np.where(assignments == j)[0]
            if members.size == 0:
                new_idx = rng.integers(N)
            else:
                intra = D[np.ix_(members, members)].sum(axis=1)
                new_idx = members[np.argmin(intra)]
            shift = D[medoid_indices[j], new_idx]
            total_shift += shift
            new_medoid_indices.append(new_idx)
        medoid_indices = new_medoid_indices
        if total_shift < tol:
            print(f"Converged in {iteration + 1} iterations with total shift {total_shift:.6f}.")
            break
    return medoid_indices


def assign(coords, medoid_coords, device: int = 0) -> np.ndarray:
    """Nearest medoid of every occurrence: argmin_j compute_rmsd(coords_i, medoid_j)
    (bpe.py:645-657, 1764-1777: P = the occurrence, Q = the medoid)."""
    return np.argmin(rmsd_cross(coords, medoid_coords, device=device), axis=1)
