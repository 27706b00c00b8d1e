"""Float64 numpy restatement of the reference's featurisation geometry
(canonical_distances_and_dihedrals, foldingdiff/angles_and_coords.py:69-154, with
biotite.structure dihedral / angle): test infrastructure for tests/test_featurize.py
and the config-1 fixture of make_golden.py."""
import numpy as np

COLUMNS = ["0C:1N", "N:CA", "CA:C", "phi", "psi", "omega", "tau", "CA:C:1N", "C:1N:1CA"]


def dihedral(p1, p2, p3, p4):  # biotite.structure.dihedral
    b1, b2, b3 = p2 - p1, p3 - p2, p4 - p3
    b1 = b1 / np.linalg.norm(b1, axis=-1, keepdims=True)
    b2 = b2 / np.linalg.norm(b2, axis=-1, keepdims=True)
    b3 = b3 / np.linalg.norm(b3, axis=-1, keepdims=True)
    n1, n2 = np.cross(b1, b2), np.cross(b2, b3)
    return np.arctan2(np.sum(np.cross(n1, n2) * b2, -1), np.sum(n1 * n2, -1))


def angle(a, b, c):  # biotite.structure.angle
    v1, v2 = a - b, c - b
    return np.arccos(np.sum(v1 * v2, -1) / (np.linalg.norm(v1, axis=-1) * np.linalg.norm(v2, axis=-1)))


def reference_columns(bb):
    """The nine columns of one chain (n, 3, 3) with the reference's index conventions."""
    n = len(bb)
    N, CA, C = bb[:, 0], bb[:, 1], bb[:, 2]
    out = {k: np.full(n, np.nan) for k in ("phi", "psi", "omega", "tau", "CA:C:1N", "C:1N:1CA")}
    out.update({k: np.zeros(n) for k in ("0C:1N", "N:CA", "CA:C")})
    if n > 1:
        out["phi"][1:] = dihedral(C[:-1], N[1:], CA[1:], C[1:])
        out["psi"][:-1] = dihedral(N[:-1], CA[:-1], C[:-1], N[1:])
        out["omega"][:-1] = dihedral(CA[:-1], C[:-1], N[1:], CA[1:])
        out["tau"][:-1] = angle(N[1:], CA[1:], C[1:])
        out["CA:C:1N"][:-1] = angle(CA[:-1], C[:-1], N[1:])
        out["C:1N:1CA"][:-1] = angle(C[:-1], N[1:], CA[1:])
        out["0C:1N"][:-1] = np.linalg.norm(N[1:] - C[:-1], axis=-1)
        out["N:CA"][:-1] = np.linalg.norm(CA[1:] - N[1:], axis=-1)
        out["CA:C"][:-1] = np.linalg.norm(C[1:] - CA[1:], axis=-1)
    return out


def pdb_dir_corpus(pdb_dir, min_length=40):
    """geobpe.pdb.load_pdb_dir's rules with the numpy geometry: sorted files, the
    backbone reader, angle range, min_length, the seed-6489 shuffle, encode.py's
    missing-dihedral filter."""
    import os
    from geobpe import pdb
    chains, names = [], []
    for f in pdb.pdb_files(pdb_dir):
        try:
            bb = pdb.backbone(f)
        except ValueError:
            continue
        if len(bb):
            chains.append(bb)
            names.append(f)
    cols = [reference_columns(bb) for bb in chains]
    keep = []
    for i, c in enumerate(cols):
        ang = [c[k] for k in ("phi", "psi", "omega", "tau", "CA:C:1N", "C:1N:1CA")]
        if any(np.nanmin(v) < -np.pi or np.nanmax(v) > np.pi for v in ang if np.any(~np.isnan(v))):
            continue
        if min_length and len(chains[i]) < min_length:
            continue
        keep.append(i)
    np.random.default_rng(seed=6489).shuffle(keep)
    keep = [i for i in keep if np.sum(~np.isnan(cols[i]["psi"])) >= len(chains[i]) - 1]
    out = {k: np.concatenate([cols[i][k] for i in keep]) for k in COLUMNS}
    out["row_off"] = np.concatenate([[0], np.cumsum([len(chains[i]) for i in keep])]).astype(np.int64)
    return out, [os.path.basename(names[i]) for i in keep]
