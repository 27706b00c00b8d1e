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


# NeRF (nerf.py:85-211 place_dihedral / NERFBuilder.cartesian_coords;
# angles_and_coords.py:232-316 update_backbone_positions), restated with numpy
N_INIT = np.array([17.047, 14.099, 3.625])
CA_INIT = np.array([16.967, 12.784, 4.338])
C_INIT = np.array([15.685, 12.755, 5.133])


def _unit(x):
    return x / np.linalg.norm(x)


def place(a, b, c, angle, length, torsion):
    bc = _unit(c - b)
    n = _unit(np.cross(b - a, bc))
    m = np.stack([bc, np.cross(n, bc), n], axis=-1)
    d = np.array([-length * np.cos(angle), length * np.cos(torsion) * np.sin(angle),
                  length * np.sin(torsion) * np.sin(angle)])
    return m @ d + c


def start(l_ca_c, l_n_ca, theta):
    ca = C_INIT + l_ca_c * _unit(CA_INIT - C_INIT)
    vn, vc = N_INIT - ca, C_INIT - ca
    cur = np.arccos(np.clip(np.dot(vn, vc) / (np.linalg.norm(vn) * np.linalg.norm(vc)), -1.0, 1.0))
    k = _unit(np.cross(vn, vc))
    ang = -(theta - cur)
    rv = vn * np.cos(ang) + np.cross(k, vn) * np.sin(ang) + k * np.dot(k, vn) * (1 - np.cos(ang))
    return ca + rv / np.linalg.norm(rv) * l_n_ca, ca, C_INIT.copy()


def nerf_packed(off, packed) -> list:
    """nerf() of spans in geobpe_nerf's packed layout (9 per residue: N:CA, CA:C, tau, 0C:1N,
    CA:C:1N, C:1N:1CA, psi, omega, phi; off[n + 1] residue offsets) -- the CPU stand-in for
    geobpe.rmsd.nerf_packed."""
    cols = ["N:CA", "CA:C", "tau", "0C:1N", "CA:C:1N", "C:1N:1CA", "psi", "omega", "phi"]
    out = []
    for a, b in zip(off[:-1], off[1:]):
        blk = np.asarray(packed[a:b])
        r = b - a
        out.append(nerf({k: list(blk[:r if c < 3 else r - 1, c]) for c, k in enumerate(cols)}))
    return out


def nerf_atoms(off, packed) -> np.ndarray:
    """nerf_packed's spans back to back, (3 * off[-1], 3) -- the CPU stand-in for
    geobpe.rmsd.nerf_atoms."""
    out = nerf_packed(off, packed)
    return np.concatenate(out).reshape(-1, 3) if out else np.zeros((0, 3))


def nerf(geo: dict) -> np.ndarray:
    """Tokenizer.geo_nerf(geo).cartesian_coords (3r - 1 bonds -> 3r atoms)."""
    r = len(geo["N:CA"])
    out = list(start(geo["CA:C"][0], geo["N:CA"][0], geo["tau"][0]))
    for i in range(r - 1):
        out.append(place(out[-3], out[-2], out[-1], geo["CA:C:1N"][i], geo["0C:1N"][i], geo["psi"][i]))
        out.append(place(out[-3], out[-2], out[-1], geo["C:1N:1CA"][i], geo["N:CA"][i + 1], geo["omega"][i]))
        out.append(place(out[-3], out[-2], out[-1], geo["tau"][i + 1], geo["CA:C"][i + 1], geo["phi"][i]))
    return np.array(out)


def k_medoids_from_matrix(D: np.ndarray, k, max_iterations: int = 10, tol: float = 1e-4, *, rng=None):
    """The host iterations of algo.k_medoids (foldingdiff/algo.py:191-213) on a given distance
    matrix, in numpy: the comparator of the product's C step (csrc/rmsdkey.c kmed_step,
    geobpe.rmsd.k_medoids_from_matrix).  The same Generator draws in the same order, the
    per-row argmin (first minimum) and each cluster's float32 member sums."""
    N = len(D)
    k = min(N, k)
    if rng is None:
        rng = np.random.default_rng(None)
    medoid_indices = rng.choice(np.arange(N), size=k, replace=False)
    for iteration in range(max_iterations):
        assignments = np.argmin(D[:, medoid_indices], axis=1)  # (all rows at once: the same values)
        total_shift = 0.0
        new_medoid_indices = []
        for j in range(k):
            members = np.where(assignments == j)[0]
            if members.size == 0:
                new_idx = rng.integers(N)
            else:
                new_idx = members[np.argmin(D[np.ix_(members, members)].sum(axis=1))]
            total_shift += D[medoid_indices[j], new_idx]
            new_medoid_indices.append(new_idx)
        medoid_indices = new_medoid_indices
        if total_shift < tol:
            break
    return medoid_indices
