"""CPU restatement of the reference's Kabsch RMSD (TEST INFRASTRUCTURE: imported
only by tests/ as the checker of csrc/rmsd.h, never by the product path).

foldingdiff/algo.py:8-46 (kabsch) and :48-65 (compute_rmsd), restated with numpy:
centre both structures, H = Pc^T Qc, SVD H = U S Vt, R = U Vt with Vt's last row
negated when det(R) < 0, Q aligned = Qc R^T + centroid(P), RMSD = sqrt(mean
squared residual).  Pinned against the reference itself by
tests/golden/rmsd_ref.npz (tests/golden/make_rmsd_golden.py).
"""
from __future__ import annotations

import numpy as np


def rmsd(P: np.ndarray, Q: np.ndarray) -> float:
    P = np.asarray(P, dtype=np.float64)
    Q = np.asarray(Q, dtype=np.float64)
    cp, cq = P.mean(axis=0), Q.mean(axis=0)
    H = (P - cp).T @ (Q - cq)
    U, _, Vt = np.linalg.svd(H)
    R = U @ Vt
    if np.linalg.det(R) < 0:
        Vt = Vt.copy()
        Vt[2, :] = -Vt[2, :]
        R = U @ Vt
    res = P - ((Q - cq) @ R.T + cp)
    return float(np.sqrt(np.mean(np.sum(res * res, axis=1))))


def rmsd_matrix(S) -> np.ndarray:
    """k_medoids' float32 matrix: upper triangle rmsd(S[i], S[j]), mirrored."""
    N = len(S)
    D = np.empty((N, N), dtype=np.float32)
    for i in range(N):
        for j in range(i, N):
            D[i, j] = D[j, i] = rmsd(S[i], S[j])
    return D
