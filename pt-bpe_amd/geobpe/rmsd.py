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
  Tokenizer.compute_coords(index, length)     compute_coords(cols, spans)  (device NeRF)
    tokenizer.py:347-363, nerf.py:85-211

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


def release_scratch(device: int = -1) -> None:
    """Free the device scratch arenas of geobpe_rmsd / geobpe_nerf / geobpe_glue_opt
    (geobpe_arena_release; -1: every device).  The next call re-creates them."""
    rc = _native.lib().geobpe_arena_release(device)
    if rc:
        raise _native.GeoBPEError(f"geobpe_arena_release failed (code {rc})")


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


def _keyc():
    from .rmsd_bpe import _KEYC
    return _KEYC


def k_medoids_from_matrix(D: np.ndarray, k, max_iterations: int = 10, tol: float = 1e-4, *, rng=None):
    """The iterations of algo.k_medoids (algo.py:191-213) on a given distance matrix: the
    assignment argmin and every cluster's member sums in C (csrc/rmsdkey.c kmed_step, numpy's
    float32 pairwise summation order and first-minimum rule, so the medoids are the reference's
    bit for bit; tests compare it with the numpy loop of oracle/rmsd.py), the Generator draws
    here in the reference's order.  The reference's matrix is float32 (algo.py:179-189): D is
    taken as float32 once, for the step and the shifts alike."""
    keyc = _keyc()
    if keyc is None:
        raise RuntimeError("the RMSD mode's C extension (_rmsdkey.so) is not built: geobpe.build.build_keys()")
    Dc = np.ascontiguousarray(D, dtype=np.float32)
    N = len(Dc)
    k = min(N, k)
    if rng is None:
        rng = np.random.default_rng(None)
    medoid_indices = rng.choice(np.arange(N), size=k, replace=False)
    asg = np.zeros(N, dtype=np.int64)
    for iteration in range(max_iterations):
        picks = keyc.kmed_step(Dc, [int(m) for m in medoid_indices], asg)
        total_shift = 0.0
        new_medoid_indices = []
        for j in range(k):
            new_idx = picks[j] if picks[j] >= 0 else rng.integers(N)  # (empty cluster, j order)
            total_shift += Dc[medoid_indices[j], new_idx]
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


# ---------------------------------------------------------------- coordinates (NeRF)
BOND_TYPES = ["N:CA", "CA:C", "0C:1N"]        # tokenizer.py:19-22
BOND_ANGLES = ["tau", "CA:C:1N", "C:1N:1CA"]
DIHEDRALS = ["psi", "omega", "phi"]
N_INIT = np.array([17.047, 14.099, 3.625])     # nerf.py:21-23 (1CRN)
CA_INIT = np.array([16.967, 12.784, 4.338])
C_INIT = np.array([15.685, 12.755, 5.133])


def init_geometry():
    """(N-CA, CA-C, N-CA-C angle) of the initial residue (Tokenizer._init_coords,
    tokenizer.py:74-77)."""
    a, b = N_INIT - CA_INIT, C_INIT - CA_INIT
    ang = float(np.arccos(np.clip(np.dot(a / np.linalg.norm(a), b / np.linalg.norm(b)), -1.0, 1.0)))
    return float(np.linalg.norm(N_INIT - CA_INIT)), float(np.linalg.norm(CA_INIT - C_INIT)), ang


def token_geo(cols: dict, idx: int, l: int, init=None) -> dict:
    """Tokenizer.token_geo(idx, l) (tokenizer.py:131-202) of one chain given its
    nine columns: bond b -> init N:CA / CA:C for b = 0, 1, else column
    BOND_TYPES[b % 3] row (b - 2) // 3; angle a -> init tau for a = 0, else
    BOND_ANGLES[a % 3] row (a - 1) // 3; dihedral d -> DIHEDRALS[d % 3] row (d + 1) // 3."""
    n_ca, ca_c, tau0 = init if init is not None else init_geometry()
    out = {}
    for j in range(idx, idx + l):
        v = n_ca if j == 0 else (ca_c if j == 1 else float(cols[BOND_TYPES[j % 3]][(j - 2) // 3]))
        out.setdefault(BOND_TYPES[j % 3], []).append(v)
    for j in range(idx, idx + l - 1):
        v = tau0 if j == 0 else float(cols[BOND_ANGLES[j % 3]][(j - 1) // 3])
        out.setdefault(BOND_ANGLES[j % 3], []).append(v)
    for j in range(idx, idx + l - 2):
        out.setdefault(DIHEDRALS[j % 3], []).append(float(cols[DIHEDRALS[j % 3]][(j + 1) // 3]))
    return out


def geo_coords(geos, device: int = 0):
    """Tokenizer.geo_nerf(geo).cartesian_coords for a batch of whole-residue geometry
    dicts (3r - 1 bonds each), on the device (csrc/rmsd.h k_nerf): [(3r, 3)]."""
    rs = []
    for g in geos:
        nb = sum(len(g.get(k, [])) for k in BOND_TYPES)
        if nb % 3 != 2:
            raise ValueError(f"geo_nerf needs 3r - 1 bonds, got {nb}")
        rs.append((nb + 1) // 3)
    off = np.zeros(len(geos) + 1, dtype=np.int64)
    np.cumsum(rs, out=off[1:])
    R = int(off[-1])
    packed = np.zeros((max(R, 1), 9), dtype=np.float64)
    for g, a, r in zip(geos, off[:-1], rs):
        blk = packed[a:a + r]
        blk[:, 0], blk[:, 1], blk[:, 2] = g["N:CA"], g["CA:C"], g["tau"]
        if r > 1:
            for c, k in enumerate(["0C:1N", "CA:C:1N", "C:1N:1CA", "psi", "omega", "phi"], start=3):
                blk[:r - 1, c] = g[k]
    return nerf_packed(off, packed, device)


def nerf_atoms(off: np.ndarray, packed: np.ndarray, device: int = 0) -> np.ndarray:
    """geobpe_nerf on spans already packed (9 float64 per residue, off[n + 1] residue
    offsets): the atoms of every span back to back, (3 * off[-1], 3)."""
    L = _native.lib()
    R = int(off[-1])
    xyz = np.empty((max(R, 1), 3, 3), dtype=np.float64)
    if R:
        rc = L.geobpe_nerf(int(device), len(off) - 1, off.ctypes.data_as(ctypes.c_void_p),
                           packed.ctypes.data_as(ctypes.c_void_p), xyz.ctypes.data_as(ctypes.c_void_p))
        if rc:
            raise _native.GeoBPEError(f"geobpe_nerf failed (code {rc})")
    return xyz.reshape(-1, 3)[:3 * R]


def nerf_packed(off: np.ndarray, packed: np.ndarray, device: int = 0):
    """nerf_atoms split per span: [(3r, 3)]."""
    xyz = nerf_atoms(off, packed, device)
    return [xyz[3 * a:3 * b] for a, b in zip(off[:-1].tolist(), off[1:].tolist())]


def compute_coords(cols: dict, spans, init=None, device: int = 0):
    """Tokenizer.compute_coords(index, length) (tokenizer.py:347-363) of one chain for
    every (index, length) in spans: the geometry rounded out to whole residues, NeRF,
    then the requested atoms."""
    n = len(cols["phi"])
    geos, cuts = [], []
    for index, length in spans:
        length = min(length, 3 * n - 1 - index)
        start = 3 * (index // 3)
        end = 3 * (((index + length - 1) + 1) // 3) + 1
        geos.append(token_geo(cols, start, end - start + 1, init))
        cuts.append((index - start, end - (index + length - 1)))
    return [c[a:len(c) - b] for c, (a, b) in zip(geo_coords(geos, device=device), cuts)]
