"""PDB -> internal coordinates (geobpe.pdb; csrc/featurize.h): the C++ backbone
reader on the CPU, the HIP featurisation on the GPU against a float64 numpy
restatement of the reference's geometry (canonical_distances_and_dihedrals,
angles_and_coords.py:69-154, biotite.structure dihedral / angle) and NeRF round
trips.  Parity against biotite itself is unpinned (biotite is not installed)."""
import os

import numpy as np
import pytest

from conftest import GOLDEN

PDB_DIR = os.path.join(GOLDEN, "pdb")  # a subset of the reference's data/vqvae_pretrain/train


import sys  # noqa: E402

sys.path.insert(0, GOLDEN)
from pdb_angles import reference_columns  # noqa: E402


def _place(a, b, c, bond, angle, torsion):
    """NeRF: atom d with |cd| = bond, angle(b, c, d) = angle, dihedral(a, b, c, d) = torsion."""
    bc = (c - b) / np.linalg.norm(c - b)
    n = np.cross(b - a, bc)
    n /= np.linalg.norm(n)
    m = np.cross(n, bc)
    d2 = np.array([-bond * np.cos(angle), bond * np.sin(angle) * np.cos(torsion), bond * np.sin(angle) * np.sin(torsion)])
    return c + d2[0] * bc + d2[1] * m + d2[2] * n


def nerf_chain(rng, n):
    """A backbone from random internal coordinates; returns (bb, the generating columns)."""
    g = {"psi": rng.uniform(-np.pi, np.pi, n), "omega": rng.normal(np.pi, 0.1, n), "phi": rng.uniform(-np.pi, np.pi, n),
         "tau": rng.normal(1.94, 0.05, n), "CA:C:1N": rng.normal(2.03, 0.04, n), "C:1N:1CA": rng.normal(2.12, 0.04, n),
         "0C:1N": rng.normal(1.33, 0.01, n), "N:CA": rng.normal(1.46, 0.01, n), "CA:C": rng.normal(1.52, 0.01, n)}
    g["omega"] = (g["omega"] + np.pi) % (2 * np.pi) - np.pi
    bb = np.zeros((n, 3, 3))
    bb[0] = [[0, 0, 0], [1.46, 0, 0], [1.46 + 1.52 * np.cos(np.pi - 1.94), 1.52 * np.sin(np.pi - 1.94), 0]]
    for r in range(n - 1):
        N, CA, C = bb[r]
        N1 = _place(N, CA, C, g["0C:1N"][r], g["CA:C:1N"][r], g["psi"][r])
        CA1 = _place(CA, C, N1, g["N:CA"][r], g["C:1N:1CA"][r], g["omega"][r])
        C1 = _place(C, N1, CA1, g["CA:C"][r], g["tau"][r], g["phi"][r + 1])
        bb[r + 1] = [N1, CA1, C1]
    return bb, g


def write_pdb(path, bb, extra=""):
    names = ["N", "CA", "C"]
    lines, k = [], 1
    for r, res in enumerate(bb):
        for a in range(3):
            x, y, z = res[a]
            lines.append(f"ATOM  {k:5d}  {names[a]:<3s} ALA A{r + 1:4d}    {x:8.3f}{y:8.3f}{z:8.3f}  1.00  0.00           "
                         f"{names[a][0]}")
            k += 1
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n" + extra)


def test_pdb_reader_backbone_roundtrip(tmp_path):
    from geobpe import pdb
    bb, _ = nerf_chain(np.random.default_rng(1), 30)
    p = str(tmp_path / "x_A.pdb")
    write_pdb(p, bb, extra="HETATM 9999  O   HOH A 900       1.000   2.000   3.000  1.00  0.00           O\nEND\n")
    got = pdb.backbone(p)
    assert got.shape == (30, 3, 3) and np.max(np.abs(got - bb)) <= 5e-4 + 1e-12


def test_pdb_reader_altloc_models_and_missing_atoms(tmp_path):
    from geobpe import pdb
    bb, _ = nerf_chain(np.random.default_rng(2), 4)
    p = str(tmp_path / "alt.pdb")
    write_pdb(p, bb)
    lines = open(p).read().splitlines()
    alt = lines[1][:16] + "B" + lines[1][17:30] + "  99.000  99.000  99.000" + lines[1][54:]
    first = lines[1][:16] + "A" + lines[1][17:]
    lines = lines[:1] + [first, alt] + lines[2:]
    model2 = ["ENDMDL", "MODEL        2"] + [l.replace("ALA", "GLY") for l in lines] + ["ENDMDL"]
    open(p, "w").write("MODEL        1\n" + "\n".join(lines + model2) + "\n")
    got = pdb.backbone(p)
    assert got.shape == (4, 3, 3) and np.allclose(got, bb, atol=5e-4)  # first altloc, first model
    q = str(tmp_path / "bad.pdb")
    write_pdb(q, bb)
    l2 = [l for l in open(q).read().splitlines() if not (" CA " in l and "A   3" in l)]
    open(q, "w").write("\n".join(l2) + "\n")
    with pytest.raises(ValueError):
        pdb.backbone(q)


def test_bundled_pdbs_parse():
    from geobpe import pdb
    for f in pdb.pdb_files(PDB_DIR):
        bb = pdb.backbone(f)
        assert len(bb) > 0
        d = np.linalg.norm(bb[:, 1] - bb[:, 0], axis=-1)  # N-CA bond
        assert 1.3 < np.median(d) < 1.6


@pytest.mark.gpu
def test_featurize_matches_numpy_reference_geometry():
    from geobpe import pdb
    chains = [pdb.backbone(f) for f in pdb.pdb_files(PDB_DIR)]
    rng = np.random.default_rng(3)
    chains += [nerf_chain(rng, n)[0] for n in (1, 2, 3, 57)]
    c = pdb.featurize(chains)
    ro = c["row_off"]
    for i, bb in enumerate(chains):
        ref = reference_columns(bb)
        for k, v in ref.items():
            got = c[k][ro[i]:ro[i + 1]]
            assert np.array_equal(np.isnan(got), np.isnan(v)), k
            m = ~np.isnan(v)
            assert np.allclose(got[m], v[m], rtol=0, atol=1e-12), k


@pytest.mark.gpu
def test_featurize_recovers_nerf_internal_coordinates():
    from geobpe import pdb
    rng = np.random.default_rng(4)
    bb, g = nerf_chain(rng, 200)
    c = pdb.featurize([bb])
    n = 200
    for k in ("psi", "omega", "CA:C:1N", "C:1N:1CA", "0C:1N", "N:CA", "CA:C", "tau"):
        assert np.allclose(c[k][: n - 1], g[k][: n - 1], atol=1e-9), k
    w = (c["phi"][1:] - g["phi"][1:] + np.pi) % (2 * np.pi) - np.pi
    assert np.max(np.abs(w)) < 1e-9 and np.isnan(c["phi"][0]) and np.isnan(c["psi"][-1])


@pytest.mark.gpu
def test_config1_pdb_corpus_trains_like_the_oracle(oracle_lib):
    """Config 1 shape (bin/encode.py on a PDB directory, 5 bins, 50 merges) on the
    bundled subset: the HIP loop on the featurised corpus equals the oracle."""
    from geobpe import pdb
    from geobpe.engine import GeoBPEEngine
    corpus, names = pdb.load_pdb_dir(PDB_DIR, min_length=40)
    assert len(names) >= 5
    o = oracle_lib.OracleBPE(corpus, 5).initialize()
    o.bin()
    for _ in range(50):
        o.step()
    e = GeoBPEEngine(corpus, 5, device=0).initialize()
    assert e.thresholds == o.thresholds
    e.bin()
    e.run(50)
    assert e.merge_keys() == o.merges
    for x, y in zip(e.encode(), o.encode()):
        assert np.array_equal(x, y)
    e.close()
