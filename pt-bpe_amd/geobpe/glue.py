"""Glue optimisation of the RMSD mode on the device.

  reference (foldingdiff/bpe.py)                    here
  _cache_exit_frames / Tokenizer.exit_frame         exit_frames: one device NeRF batch for every
    (:700-705, tokenizer.py:458-477)                  chain, frame_from_triad on the host
  glue_opt_all / _opt_glue_worker / opt_glue        optimize_chains: one geobpe_glue_opt launch
    (:106-135, :739-807)                              for all chains (csrc/glue.h, one chain per
  optimize_glues_entry_torch / fk_segment_torch       thread: NeRF, frame loss, prior, reverse
    (:423-578)                                        sweep and the L-BFGS control flow)
  snap_bin (:495-524)                               snap_bin, on the host

The product path has no CPU fallback: ``_native.lib()`` raises if libgeobpe.so is missing.
"""
from __future__ import annotations

import bisect
import ctypes

import numpy as np

from . import _native
from . import rmsd as _rmsd

GLUE = ["omega", "C:1N:1CA", "phi"]


def pack_chain(cur: dict, init) -> np.ndarray:
    """The chain's geometry in the device layout (geobpe_nerf): per residue k,
    {N:CA_k, CA:C_k, tau_k, 0C:1N_k, CA:C:1N_k, C:1N:1CA_k, psi_k, omega_k, phi_{k+1}}
    (Tokenizer.token_geo(0, 3n-1) index rules, tokenizer.py:169-202), rounded to float32 as
    fk_segment_torch's torch.as_tensor(..., dtype=float32) does (bpe.py:427-428)."""
    n = len(cur["phi"])
    g = np.zeros((n, 9), dtype=np.float64)
    g[0, :3] = init
    col = lambda c: np.asarray(cur[c], dtype=np.float64)  # noqa: E731
    if n > 1:
        g[1:, 0] = col("N:CA")[:n - 1]
        g[1:, 1] = col("CA:C")[:n - 1]
        g[1:, 2] = col("tau")[:n - 1]
        for j, c in enumerate(["0C:1N", "CA:C:1N", "C:1N:1CA", "psi", "omega"], start=3):
            g[:n - 1, j] = col(c)[:n - 1]
        g[:n - 1, 8] = col("phi")[1:n]
    return g.astype(np.float32).astype(np.float64)


def frame_from_triad(N, CA, C):
    """angles_and_coords.py:571-583 (numpy, eps 1e-12), batched over residues."""
    def norm(v):
        return v / (np.linalg.norm(v, axis=-1, keepdims=True) + 1e-12)
    x = norm(C - CA)
    u = norm(N - CA)
    z = norm(np.cross(x, u))
    y = np.cross(z, x)
    return np.stack([x, y, z], axis=-1), CA.copy()


def exit_frames(chains, device: int = 0):
    """Tokenizer.exit_frame(3, 3n-4, ret_all=True) for every chain (bpe.py:700-705): the
    frames of residues 0..n-2 of the chain's NeRF (compute_coords(0, 3n-1)).  [(R (n-1,3,3),
    t (n-1,3))]; one device NeRF batch."""
    geos = [_rmsd.token_geo(c.cur, 0, 3 * c.n - 1, tuple(c.init)) for c in chains]
    out = []
    for xyz in _rmsd.geo_coords(geos, device=device):
        r = len(xyz) // 3
        a = xyz.reshape(r, 3, 3)[:r - 1]
        out.append(frame_from_triad(a[:, 0], a[:, 1], a[:, 2]))
    return out


def optimize_chains(geos, x0s, targets, grids, prior, lam: float, device: int = 0, w_rot=1.0, w_trans=0.1):
    """One geobpe_glue_opt launch.  geos: [(r, 9)] from pack_chain; x0s: [(r-1, 3)] start
    glues; targets: [(R (r-1,3,3), t (r-1,3))]; grids: prior table index per chain; prior:
    (n_grid, 3, 2, kmax) float32 centres / weights and (n_grid, 3) counts.  Returns the
    wrapped optimum [(r-1, 3) float32], (iterations, evaluations) and (first, last loss) per
    chain."""
    L = _native.lib()
    n = len(geos)
    rs = [len(g) for g in geos]
    if any(r < 1 for r in rs):
        raise ValueError("glue opt: a chain with no residues")
    off = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(rs, out=off[1:])
    geo = np.ascontiguousarray(np.concatenate(geos) if n else np.zeros((0, 9)), dtype=np.float64)
    ng = int(off[-1]) - n
    x0 = np.ascontiguousarray(np.concatenate([np.asarray(x, dtype=np.float32).reshape(-1, 3) for x in x0s])
                              if ng else np.zeros((0, 3), np.float32))
    tg = np.zeros((max(ng, 1), 12), dtype=np.float32)
    p = 0
    for (R, t), r in zip(targets, rs):
        m = r - 1
        if len(R) < m:
            raise ValueError(f"glue opt: {len(R)} target frames for {m} glues")
        tg[p:p + m, :9] = np.asarray(R[:m], dtype=np.float32).reshape(m, 9)
        tg[p:p + m, 9:] = np.asarray(t[:m], dtype=np.float32)
        p += m
    table, counts = prior
    table = np.ascontiguousarray(table, dtype=np.float32)
    counts = np.ascontiguousarray(counts, dtype=np.int32)
    grid = np.ascontiguousarray(grids, dtype=np.int32)
    xout = np.zeros((max(ng, 1), 3), dtype=np.float32)
    stats = np.zeros((max(n, 1), 2), dtype=np.int32)
    loss = np.zeros((max(n, 1), 2), dtype=np.float64)
    if ng > 0:
        vp = ctypes.c_void_p
        rc = L.geobpe_glue_opt(int(device), n, off.ctypes.data_as(vp), geo.ctypes.data_as(vp), x0.ctypes.data_as(vp),
                               tg.ctypes.data_as(vp), grid.ctypes.data_as(vp), int(table.shape[0]),
                               int(table.shape[-1]), table.ctypes.data_as(vp), counts.ctypes.data_as(vp),
                               float(lam), float(w_rot), float(w_trans), xout.ctypes.data_as(vp),
                               stats.ctypes.data_as(vp), loss.ctypes.data_as(vp))
        if rc:
            raise _native.GeoBPEError(f"geobpe_glue_opt failed (code {rc})")
    outs, p = [], 0
    for r in rs:
        outs.append(xout[p:p + r - 1].copy())
        p += r - 1
    return outs, stats[:n], loss[:n]


def prior_tables(grids_thr, grids_counts):
    """_bin_centers / _bin_weights (bpe.py:834-872) of each grid as device tables: centres
    = float32 mean of each bin's edges, weights = float32 counts / their sum, for omega,
    C:1N:1CA and phi."""
    kmax = max(len(thr[k]) for thr in grids_thr for k in GLUE)
    table = np.zeros((len(grids_thr), 3, 2, kmax), dtype=np.float32)
    counts = np.zeros((len(grids_thr), 3), dtype=np.int32)
    for gi, (thr, cnt) in enumerate(zip(grids_thr, grids_counts)):
        for t, k in enumerate(GLUE):
            e = np.asarray(thr[k], dtype=np.float32)
            c = np.asarray(cnt[k], dtype=np.float32)
            table[gi, t, 0, :len(e)] = e.mean(axis=-1)
            table[gi, t, 1, :len(c)] = c / np.float32(sum(cnt[k]))
            counts[gi, t] = len(e)
    return table, counts


def snap_bin(arr, x):
    """snap_bin (bpe.py:495-524) on the float32 optimum: the first edge below the range, the
    last edge at or above it, else the centre of the bin found by bisect_right over the right
    edges (compared in float32, as the reference compares its float32 tensor)."""
    x = np.float32(x)
    if x < np.float32(arr[0][0]):
        return arr[0][0]
    if x >= np.float32(arr[-1][1]):
        return arr[-1][1]
    i = bisect.bisect_right([np.float32(b) for _, b in arr], x)
    return sum(arr[i]) / 2


def snap_many(arr, xs) -> np.ndarray:
    """snap_bin over an array of optima (same float32 comparisons, numpy searchsorted with
    side="right" = bisect_right)."""
    xs = np.asarray(xs, dtype=np.float32)
    right = np.array([np.float32(b) for _, b in arr], dtype=np.float32)
    centre = np.array([sum(e) / 2 for e in arr], dtype=np.float64)
    i = np.minimum(np.searchsorted(right, xs, side="right"), len(arr) - 1)
    out = centre[i]
    out = np.where(xs < np.float32(arr[0][0]), arr[0][0], out)
    return np.where(xs >= np.float32(arr[-1][1]), arr[-1][1], out)
