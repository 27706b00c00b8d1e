"""Golden vectors for the RMSD partitioning primitives,
made by running the REFERENCE's foldingdiff/algo.py in this container.

Writes ``tests/golden/rmsd_ref.npz``:
  A (48, 10, 3)       backbone-like chains: random walks, rigid copies of some
                      (RMSD ~ 0) and mirror images of some (the reflection case)
  B (8, 10, 3)        more chains (the "medoids" of the cross matrix)
  D_ref (48, 48)      k_medoids' float32 distance matrix (algo.py:179-189 loop)
  cross_ref (48, 8)   compute_rmsd(A_i, B_j) (algo.py:48-65), float64
  medoids_ref (5,)    algo.k_medoids(A, 5, rng=default_rng(3))
  A3 (30, 3, 3), D3_ref, medoids3_ref (4,)   three-atom structures (one residue's
                      N, CA, C), k = 4, rng=default_rng(5)
  nerf_*              Tokenizer.compute_coords(index, length) (tokenizer.py:347-363,
                      NeRF) of spans of five synthetic chains (1..30 residues):
                      the chains' nine columns + row_off, spans (chain, index,
                      length), the coordinates concatenated + their offsets
Usage:  python tests/golden/make_rmsd_golden.py
"""
from __future__ import annotations

import io
import os
import sys
from contextlib import redirect_stdout

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def chains(rng, n, atoms):
    out = np.empty((n, atoms, 3))
    for s in range(n):
        x = np.zeros((atoms, 3))
        d = rng.normal(size=3)
        for a in range(1, atoms):
            d = 0.6 * d / np.linalg.norm(d) + 0.8 * rng.normal(size=3)
            x[a] = x[a - 1] + 1.45 * d / np.linalg.norm(d)
        out[s] = x
    return out


def rotation(rng):
    q = rng.normal(size=4)
    q /= np.linalg.norm(q)
    w, x, y, z = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


def nerf_fixture() -> dict:
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(HERE)), "pt-bpe_amd"))
    sys.path.insert(0, HERE)
    import make_golden
    from geobpe import synth
    make_golden._stub_optional_deps()
    from foldingdiff.tokenizer import Tokenizer

    lengths = np.array([1, 2, 7, 15, 30])
    corpus = synth.make_corpus(lengths, seed=12)
    spans, coords, coff = [], [], [0]
    for ci, row in enumerate(synth.corpus_rows(corpus)):
        n = len(row["phi"])
        s = Tokenizer.init_structure(n)
        for c in synth.COLUMNS:
            s["angles"][c] = row[c].astype(np.float64)
        s["fname"] = f"synthetic_{ci}"
        t = Tokenizer(s)
        cand = [(0, 3 * n - 1), (0, 3), (0, 2), (3, 6), (3 * (n - 1), 2), (3, 3 * (n - 2)), (6, 9), (4, 5)]
        for index, length in cand:
            if index < 0 or length <= 0 or index + length > 3 * n - 1:
                continue
            xyz = np.asarray(t.compute_coords(index, length), dtype=np.float64)
            spans.append((ci, index, length))
            coords.append(xyz)
            coff.append(coff[-1] + len(xyz))
    return {**{f"nerf_{k}": v for k, v in corpus.items()}, "nerf_spans": np.array(spans, dtype=np.int64),
            "nerf_coords": np.concatenate(coords), "nerf_coff": np.array(coff, dtype=np.int64)}


def main():
    sys.path.insert(0, "/root/reference")
    from foldingdiff import algo

    rng = np.random.default_rng(2024)
    A = chains(rng, 48, 10)
    for s in range(0, 12, 3):  # rigid copies: RMSD ~ 0 to their source
        A[s + 1] = A[s] @ rotation(rng).T + rng.normal(size=3) * 5
    for s in range(12, 20, 2):  # mirror images (det -1): the reflection correction matters
        A[s + 1] = A[s] * np.array([-1.0, 1.0, 1.0]) + rng.normal(size=3)
    A[30:36] = A[24] + rng.normal(scale=0.05, size=(6, 10, 3))  # a tight cluster
    B = chains(rng, 8, 10)
    B[0] = A[5] @ rotation(rng).T

    def dmat(S):
        N = len(S)
        D = np.empty((N, N), dtype=np.float32)
        for i in range(N):
            for j in range(i, N):
                D[i, j] = D[j, i] = algo.compute_rmsd(S[i], S[j])
        return D

    D_ref = dmat(A)
    cross_ref = np.array([[algo.compute_rmsd(a, b) for b in B] for a in A])
    A3 = chains(rng, 30, 3)
    A3[1] = A3[0] @ rotation(rng).T
    D3_ref = dmat(A3)
    with redirect_stdout(io.StringIO()):
        med = algo.k_medoids(list(A), 5, rng=np.random.default_rng(3))
        med3 = algo.k_medoids(list(A3), 4, rng=np.random.default_rng(5))
    nerf = nerf_fixture()
    np.savez_compressed(os.path.join(HERE, "rmsd_ref.npz"), A=A, B=B, D_ref=D_ref, cross_ref=cross_ref,
                        medoids_ref=np.array(med, dtype=np.int64), A3=A3, D3_ref=D3_ref,
                        medoids3_ref=np.array(med3, dtype=np.int64), **nerf)
    print("medoids", list(map(int, med)), "medoids3", list(map(int, med3)))


if __name__ == "__main__":
    main()
