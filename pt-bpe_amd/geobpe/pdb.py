"""PDB structures -> the internal-coordinate corpus of the GeoBPE loop
(config 1: scripts/encode.sh on data/vqvae_pretrain/train).

The reference featurises with biotite (``canonical_distances_and_dihedrals``,
foldingdiff/angles_and_coords.py:69-154) inside ``FullCathCanonicalCoordsDataset``
(foldingdiff/datasets.py:194-331) and bin/encode.py drops chains with missing
dihedrals (bin/encode.py:276-283).  Here:

  * ``geobpe_pdb_backbone`` (C++, csrc/featurize.h) reads N / CA / C of every
    amino-acid residue of the first model (first alternate location); a residue
    missing one of them makes the file unusable (biotite's BadStructureError);
  * ``geobpe_featurize`` (HIP, one thread per residue) computes the nine columns
    with the reference's index conventions (header of csrc/featurize.h);
  * ``load_pdb_dir`` applies the dataset's rules: ``.pdb`` / ``.pdb.gz`` files of
    a directory, ``toy`` first files, angles within [-pi, pi], ``min_length``
    residues, the seed-6489 shuffle (datasets.py:286-288), and encode.py's
    missing-dihedral filter.  The file order before the shuffle is sorted by name
    (the reference uses unsorted glob order, which depends on the filesystem).

Parity against biotite is UNPINNED in this build (biotite is not installed):
tests check the device geometry against a float64 numpy restatement and NeRF
round trips.  Values that land within rounding of a histogram edge could bin
differently from the reference's.
"""
from __future__ import annotations

import ctypes
import gzip
import os
import tempfile

import numpy as np

from . import _native
from .synth import COLUMNS


def backbone(path: str) -> np.ndarray:
    """(n, 3, 3) float64: N, CA, C coordinates per residue."""
    L = _native.lib()
    src = path
    tmp = None
    if path.endswith(".gz"):  # the C++ reader takes plain text
        with gzip.open(path, "rb") as f:
            data = f.read()
        tmp = tempfile.NamedTemporaryFile(suffix=".pdb", delete=False)
        tmp.write(data)
        tmp.close()
        src = tmp.name
    try:
        n = L.geobpe_pdb_backbone(src.encode(), None, 0)
        if n < 0:
            msg = L.geobpe_pdb_error().decode()
            raise ValueError(f"{path}: {msg}")
        xyz = np.empty((n, 3, 3), dtype=np.float64)
        if n:
            m = L.geobpe_pdb_backbone(src.encode(), xyz.ctypes.data_as(ctypes.c_void_p), n)
            if m != n:
                raise ValueError(f"{path}: {L.geobpe_pdb_error().decode()}")
        return xyz
    finally:
        if tmp is not None:
            os.unlink(tmp.name)


def featurize(chains, device: int = 0) -> dict:
    """Backbones [(n_i, 3, 3)] -> corpus {column: float64[R]} + row_off, on the GPU."""
    L = _native.lib()
    lens = [len(c) for c in chains]
    ro = np.zeros(len(chains) + 1, dtype=np.int64)
    np.cumsum(lens, out=ro[1:])
    R = int(ro[-1])
    xyz = np.ascontiguousarray(np.concatenate(chains) if chains else np.zeros((0, 3, 3)), dtype=np.float64)
    # GEOBPE_COL_* order == geobpe.synth.COLUMNS
    cols = [np.empty(R, dtype=np.float64) for _ in COLUMNS]
    ptrs = (ctypes.c_void_p * 9)(*[c.ctypes.data for c in cols])
    rc = L.geobpe_featurize(int(device), len(chains), ro.ctypes.data_as(ctypes.c_void_p),
                            xyz.ctypes.data_as(ctypes.c_void_p), ptrs)
    if rc:
        raise _native.GeoBPEError(f"geobpe_featurize failed (code {rc})")
    out = dict(zip(COLUMNS, cols))
    out["row_off"] = ro
    return out


def pdb_files(data_dir: str):
    fn = [os.path.join(data_dir, f) for f in os.listdir(data_dir) if f.endswith(".pdb") or f.endswith(".pdb.gz")]
    if not fn:
        raise FileNotFoundError(f"No PDB files found in {data_dir}")
    return sorted(fn)


def load_pdb_dir(data_dir: str, toy: int = 0, min_length: int = 40, device: int = 0, shuffle: bool = True):
    """(corpus, fnames) of a directory of PDB files with the dataset's rules."""
    fnames = pdb_files(data_dir)
    if toy:
        fnames = fnames[:toy]
    chains, names = [], []
    for f in fnames:
        try:
            bb = backbone(f)
        except ValueError:
            continue  # featurize_one returns None (datasets.py:108-164)
        if len(bb) == 0:
            continue
        chains.append(bb)
        names.append(f)
    corpus = featurize(chains, device=device)
    ro = corpus["row_off"]
    keep = []
    for i in range(len(chains)):
        a, b = int(ro[i]), int(ro[i + 1])
        ang = [corpus[k][a:b] for k in ("phi", "psi", "omega", "tau", "CA:C:1N", "C:1N:1CA")]
        if any(np.nanmin(v) < -np.pi or np.nanmax(v) > np.pi for v in ang if np.any(~np.isnan(v))):
            continue  # "Illegal values" (angles_and_coords.py:120-124)
        if min_length and b - a < min_length:
            continue  # datasets.py:263-270
        keep.append(i)
    if shuffle:  # datasets.py:286-288
        rng = np.random.default_rng(seed=6489)
        rng.shuffle(keep)
    keep = [i for i in keep if np.sum(~np.isnan(corpus["psi"][ro[i]:ro[i + 1]])) >= (ro[i + 1] - ro[i]) - 1]
    out = {k: np.concatenate([corpus[k][ro[i]:ro[i + 1]] for i in keep]) if keep else np.zeros(0)
           for k in COLUMNS}
    out["row_off"] = np.concatenate([[0], np.cumsum([ro[i + 1] - ro[i] for i in keep])]).astype(np.int64)
    return out, [names[i] for i in keep]
