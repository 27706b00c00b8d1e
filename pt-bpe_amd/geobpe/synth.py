"""Synthetic backbone internal-coordinate corpora.

The reference featurises PDB files with biotite
(`foldingdiff/angles_and_coords.py:69-154`) into a 9-column table per chain.
biotite is absent here, so the bench and the golden fixtures use synthetic
tables of the same layout:

* columns (`COLUMNS`) in the reference's `Tokenizer.init_structure` order
  (`foldingdiff/tokenizer.py:393-405`);
* row ``r`` of a chain holds residue ``r``'s values; the reference's padding is
  reproduced: ``phi[0]`` is NaN, ``psi/omega/tau/CA:C:1N/C:1N:1CA[n-1]`` are
  NaN and the three distances at ``n-1`` are 0 (`angles_and_coords.py:101-149`).

A corpus is a dict ``{column: float64[R]}`` of the chains concatenated plus
``row_off`` (int64[N+1]).  Everything is drawn from
``numpy.random.default_rng(seed)``, so a (seed, lengths) pair fixes the corpus.
"""
from __future__ import annotations

import numpy as np

COLUMNS = ["0C:1N", "N:CA", "CA:C", "phi", "psi", "omega", "tau", "CA:C:1N", "C:1N:1CA"]
ANGLE_COLUMNS = ["phi", "psi", "omega", "tau", "CA:C:1N", "C:1N:1CA"]
DIST_COLUMNS = ["0C:1N", "N:CA", "CA:C"]


def _wrap(v: np.ndarray) -> np.ndarray:
    """Wrap radians to (-pi, pi]."""
    w = np.mod(v + np.pi, 2 * np.pi) - np.pi
    w[w == -np.pi] = np.pi
    return w


def make_lengths(n_seqs: int, lo: int, hi: int | None = None, seed: int = 0) -> np.ndarray:
    """Chain lengths: all ``lo`` when ``hi`` is None, else U{lo..hi}."""
    if hi is None:
        return np.full(n_seqs, lo, dtype=np.int64)
    rng = np.random.default_rng(seed + 7919)
    return rng.integers(lo, hi + 1, size=n_seqs).astype(np.int64)


def make_corpus(lengths, seed: int = 0, repeat_frac: float = 0.0) -> dict:
    """Generate a synthetic angle corpus with the §8(d) distributions.

    ``repeat_frac`` > 0 turns that fraction of chains into near-ideal helices
    (noise 1e-3) so that long runs of identical residue symbols occur; this
    exercises the greedy run-parity rule of `BPE.step` (`bpe.py:1888-1916`).
    """
    lengths = np.asarray(lengths, dtype=np.int64)
    n = int(lengths.sum())
    rng = np.random.default_rng(seed)
    helix = rng.random(n) < 0.5
    phi = np.where(helix, rng.normal(-1.1, 0.2, n), rng.normal(-2.1, 0.3, n))
    psi = np.where(helix, rng.normal(-0.8, 0.2, n), rng.normal(2.2, 0.3, n))
    cols = {
        "phi": _wrap(phi),
        "psi": _wrap(psi),
        "omega": _wrap(rng.normal(np.pi, 0.08, n)),
        "tau": rng.normal(1.94, 0.05, n),
        "CA:C:1N": rng.normal(2.03, 0.04, n),
        "C:1N:1CA": rng.normal(2.12, 0.04, n),
        "0C:1N": rng.normal(1.33, 0.01, n),
        "N:CA": rng.normal(1.46, 0.01, n),
        "CA:C": rng.normal(1.52, 0.01, n),
    }
    row_off = np.zeros(len(lengths) + 1, dtype=np.int64)
    np.cumsum(lengths, out=row_off[1:])
    if repeat_frac > 0:
        rep = rng.random(len(lengths)) < repeat_frac
        for i in np.nonzero(rep)[0]:
            a, b = row_off[i], row_off[i + 1]
            m = b - a
            cols["phi"][a:b] = -1.0 + rng.normal(0, 1e-3, m)
            cols["psi"][a:b] = -0.75 + rng.normal(0, 1e-3, m)
            cols["omega"][a:b] = _wrap(np.pi + rng.normal(0, 1e-3, m))
            cols["tau"][a:b] = 1.94 + rng.normal(0, 1e-3, m)
            cols["CA:C:1N"][a:b] = 2.03 + rng.normal(0, 1e-3, m)
            cols["C:1N:1CA"][a:b] = 2.12 + rng.normal(0, 1e-3, m)
    first = row_off[:-1]
    last = row_off[1:] - 1
    cols["phi"][first] = np.nan
    for c in ("psi", "omega", "tau", "CA:C:1N", "C:1N:1CA"):
        cols[c][last] = np.nan
    for c in DIST_COLUMNS:
        cols[c][last] = 0.0
    out = {c: np.ascontiguousarray(cols[c], dtype=np.float64) for c in COLUMNS}
    out["row_off"] = row_off
    return out


def corpus_rows(corpus: dict):
    """Yield per-chain ``{column: float64[n]}`` views (for the reference harness)."""
    ro = corpus["row_off"]
    for i in range(len(ro) - 1):
        a, b = int(ro[i]), int(ro[i + 1])
        yield {c: corpus[c][a:b] for c in COLUMNS}


def save_corpus(path: str, corpus: dict) -> None:
    np.savez_compressed(path, **corpus)


def load_corpus(path: str) -> dict:
    with np.load(path, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}
