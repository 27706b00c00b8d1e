"""How far the device glue optimiser (csrc/glue.h) lands from the reference's own optimiser
(oracle/glue.py, bit-exact with it on the fixtures), over many chains.

  python tools/glue_drift.py oracle OUT.npz [N]   (CPU: problems + the oracle's optimum)
  python tools/glue_drift.py device OUT.npz       (GPU box: device optimum vs the saved one;
                                                   tests/golden/glue_drift_oracle.npz holds N = 120;
                                                   GEOBPE_LIB selects an A/B build)

Problems: N synthetic chains (geobpe.synth, seed 5, 20..40 residues), std bond lengths;
targets = the exit frames of the chain; start = the glue angles snapped to 5 histogram
bins (what glue_opt_all starts from), prior off.  Printed: drift quantiles (rad), the share
of glues that snap to the same bin, and the final-loss ratio quantiles.
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(REPO, "pt-bpe_amd"))
sys.path.insert(0, REPO)
GLUE_COLS = ["omega", "C:1N:1CA", "phi"]


def problems(n):
    from geobpe import glue, rmsd, synth
    from geobpe.bpe import BOND_LENGTHS
    corpus = synth.make_corpus(synth.make_lengths(n, 20, 40, seed=5), seed=5)
    ro = corpus["row_off"]
    thr = []
    for k in GLUE_COLS:
        v = np.asarray(corpus[k], dtype=np.float64)
        v = (v[~np.isnan(v)] + 2 * np.pi) % (2 * np.pi)
        e = np.histogram_bin_edges(v, bins=5)
        thr.append([(float(a), float(b)) for a, b in zip(e[:-1], e[1:])])
    geos, x0s, R, T = [], [], [], []
    init = list(rmsd.init_geometry())
    init[0], init[1] = BOND_LENGTHS[0], BOND_LENGTHS[1]
    for r in range(n):
        cols = {c: np.array(corpus[c][ro[r]:ro[r + 1]], dtype=np.float64) for c in synth.COLUMNS}
        m = len(cols["phi"])
        for i, bt in enumerate(["N:CA", "CA:C", "0C:1N"]):
            cols[bt][:m - 1] = BOND_LENGTHS[i]
        g = rmsd.token_geo(cols, 0, 3 * m - 1, tuple(init))
        xyz = rmsd_nerf(g).reshape(m, 3, 3)[:m - 1]
        Rr, tr = glue.frame_from_triad(xyz[:, 0], xyz[:, 1], xyz[:, 2])
        geo = glue.pack_chain(cols, init)
        x0 = geo[:m - 1][:, [7, 5, 8]].copy()
        for t in range(3):
            x0[:, t] = [glue.snap_bin(thr[t], (v + 2 * np.pi) % (2 * np.pi)) for v in x0[:, t]]
        geo[:m - 1][:, [7, 5, 8]] = x0
        geos.append(geo)
        x0s.append(x0.astype(np.float32))
        R.append(Rr)
        T.append(tr)
    return geos, x0s, R, T, thr


def rmsd_nerf(g):
    from oracle import rmsd as orm
    return orm.nerf(g)


def main(argv):
    mode, path = argv[0], argv[1]
    if mode == "oracle":
        from oracle import glue as og
        n = int(argv[2]) if len(argv) > 2 else 100
        geos, x0s, R, T, thr = problems(n)
        opt, loss = [], []
        for g, x0, r, t in zip(geos, x0s, R, T):
            o = og.optimize(g, x0, r, t)
            opt.append(o[0])
            loss.append(o[4])
        np.savez_compressed(path, n=n, opt=np.concatenate(opt), loss=np.array(loss))
        print(f"oracle: {n} chains saved to {path}")
        return
    print(json.dumps(device_stats(path)))


def device_stats(path):
    """The device optimum against the oracle's saved one: drift quantiles (rad), the share of
    glues snapping to the same bin, final-loss ratio quantiles."""
    from geobpe import glue
    z = np.load(path)
    geos, x0s, R, T, thr = problems(int(z["n"]))
    prior = (np.zeros((1, 3, 2, 1), np.float32), np.ones((1, 3), np.int32))
    outs, stats, loss = glue.optimize_chains(geos, x0s, list(zip(R, T)), [0] * len(geos), prior, 0.0)
    dev = np.concatenate(outs).astype(np.float64)
    ref = z["opt"].astype(np.float64)
    d = np.abs(dev - ref)
    d = np.minimum(d, 2 * np.pi - d).ravel()
    same = np.array([[glue.snap_bin(thr[t], a[t]) == glue.snap_bin(thr[t], b[t]) for t in range(3)]
                     for a, b in zip(dev, ref)])
    lr = loss[:, 1] / z["loss"]
    out = {"lib": os.environ.get("GEOBPE_LIB", "libgeobpe.so"), "chains": int(z["n"]), "glues": int(len(dev)),
           "drift_rad": {q: float(np.quantile(d, p)) for q, p in (("p50", .5), ("p90", .9), ("p99", .99), ("max", 1.0))},
           "same_bin": float(same.mean()), "loss_ratio": {"min": float(lr.min()), "p50": float(np.median(lr)),
                                                           "max": float(lr.max())}}
    return out


if __name__ == "__main__":
    main(sys.argv[1:])
