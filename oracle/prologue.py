"""numpy restatement of the reference's threshold + residue-token prologue.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

* `thresholds`   BPE._init_thresholds (foldingdiff/bpe.py:820-876) with
                 save_histogram (foldingdiff/plotting.py:305-337): per angle type,
                 every non-NaN non-zero value of the column (bpe.py:844) plus the
                 tokenizer's init N-CA-C angle for tau (bpe.py:845-846), wrapped
                 (v+2pi)%2pi, np.histogram(bins=B) edges -> [(start, end)].
* `get_ind`      BPE.get_ind (bpe.py:1164-1189): bisect_right on the left edges,
                 last right edge inclusive, ValueError otherwise.
* `symbols`      the residue / junction symbols of SURVEY.md Appendix A using the
                 Tokenizer index maps (tokenizer.py:131-167):
                 tau_j = df.tau[j-1] (j>=1; j=0 is the init angle),
                 CA:C:1N_j = df["CA:C:1N"][j], psi_j = df.psi[j],
                 omega_j = df.omega[j], C:1N:1CA_j = df["C:1N:1CA"][j],
                 phi_{j+1} = df.phi[j+1].
* `init_labels`  _init_res_tokens (bpe.py:231-261): label = first-appearance rank
                 of the residue key over (tokenizer, residue) order.
"""
from __future__ import annotations

import bisect

import numpy as np

ANGLE_TYPES = ["tau", "CA:C:1N", "C:1N:1CA", "psi", "omega", "phi"]  # Tokenizer.BOND_ANGLES + DIHEDRAL_ANGLES
# nerf.py:22-24 (init coords from 1CRN)
N_INIT = np.array([17.047, 14.099, 3.625])
CA_INIT = np.array([16.967, 12.784, 4.338])
C_INIT = np.array([15.685, 12.755, 5.133])


def init_bond_angle() -> float:
    """Tokenizer._init_coords (tokenizer.py:74-77) via angle_between (angles_and_coords.py:746-752)."""
    v1, v2 = N_INIT - CA_INIT, C_INIT - CA_INIT
    u1 = v1 / np.linalg.norm(v1)
    u2 = v2 / np.linalg.norm(v2)
    return float(np.arccos(np.clip(np.dot(u1, u2), -1.0, 1.0)))


def thresholds(corpus: dict, B: int, cover: bool = False, strategy: str = None) -> dict:
    """``cover``: bin_strategy "histogram-cover" -> range=(0, 2pi) (plotting.py:319);
    ``strategy="uniform"``: equal-count edges, np.quantile of the sorted values
    (save_histogram_equal_counts / equal_count_bin_edges, plotting.py:256-302)."""
    n_rows = len(corpus["row_off"]) - 1
    init = init_bond_angle()
    out = {}
    for key in ANGLE_TYPES:
        col = corpus[key]
        vals = col[(np.nan_to_num(col, nan=0.0) != 0.0)]
        if key == "tau":
            vals = np.concatenate([vals, np.full(n_rows, init)])
        a = (vals + 2 * np.pi) % (2 * np.pi)
        if strategy == "uniform":
            edges = np.quantile(np.sort(a), np.linspace(0, 1, B + 1))
        else:
            _, edges = np.histogram(a, bins=B, range=(0, 2 * np.pi) if cover else None)
        out[key] = [(float(s), float(e)) for s, e in zip(edges[:-1], edges[1:])]
    return out


def get_ind(v: float, values) -> int:
    left = [s for s, _ in values]
    ind = bisect.bisect_right(left, v) - 1
    if ind < 0:
        raise ValueError(f"value {v} is below the first bin range")
    s, e = values[ind]
    if ind == len(values) - 1 and v == e:
        return ind
    if s <= v < e:
        return ind
    raise ValueError(f"value {v} does not fall into any bin")


def get_ind_vec(v: np.ndarray, values) -> np.ndarray:
    """Vectorised get_ind with identical semantics (ValueError on any miss)."""
    left = np.array([s for s, _ in values])
    right = np.array([e for _, e in values])
    v = np.asarray(v, dtype=np.float64)
    ind = np.searchsorted(left, v, side="right") - 1
    bad = ind < 0
    indc = np.clip(ind, 0, len(values) - 1)
    s, e = left[indc], right[indc]
    ok = (~bad) & (((s <= v) & (v < e)) | ((indc == len(values) - 1) & (v == e)))
    if not np.all(ok):
        j = int(np.nonzero(~ok)[0][0])
        raise ValueError(f"value {v[j]} does not fall into any bin")
    return indc.astype(np.int64)


def wrap(v):
    return (v + 2 * np.pi) % (2 * np.pi)


def symbols(corpus: dict, thr: dict, B: int):
    """Residue symbols rsym[R] and junction symbols gsym[R] (gsym[j] = junction j->j+1,
    -1 at a chain's last residue)."""
    ro = corpus["row_off"]
    R = int(ro[-1])
    first = np.zeros(R, dtype=bool)
    last = np.zeros(R, dtype=bool)
    first[ro[:-1][ro[:-1] < ro[1:]]] = True
    last[(ro[1:] - 1)[ro[:-1] < ro[1:]]] = True
    tau_src = np.empty(R)
    tau_src[1:] = corpus["tau"][:-1]
    tau_src[first] = init_bond_angle()
    tau = get_ind_vec(wrap(tau_src), thr["tau"])
    nl = ~last
    cac1n = np.zeros(R, dtype=np.int64)
    psi = np.zeros(R, dtype=np.int64)
    cac1n[nl] = get_ind_vec(wrap(corpus["CA:C:1N"][nl]), thr["CA:C:1N"])
    psi[nl] = get_ind_vec(wrap(corpus["psi"][nl]), thr["psi"])
    rsym = np.where(last, B ** 3 + tau, tau * B * B + cac1n * B + psi)
    gsym = np.full(R, -1, dtype=np.int64)
    idx = np.nonzero(nl)[0]
    om = get_ind_vec(wrap(corpus["omega"][idx]), thr["omega"])
    cn = get_ind_vec(wrap(corpus["C:1N:1CA"][idx]), thr["C:1N:1CA"])
    ph = get_ind_vec(wrap(corpus["phi"][idx + 1]), thr["phi"])
    gsym[idx] = om * B * B + cn * B + ph
    return rsym.astype(np.int32), gsym.astype(np.int32)


def init_labels(rsym: np.ndarray):
    """First-appearance ranks of the residue symbols; returns (labels[R], symbol_of_label[K0])."""
    uniq, first_idx, inv = np.unique(rsym, return_index=True, return_inverse=True)
    order = np.argsort(first_idx, kind="stable")
    rank = np.empty(len(uniq), dtype=np.int64)
    rank[order] = np.arange(len(uniq))
    return rank[inv].astype(np.int32), uniq[order].astype(np.int32)


def centre(values, ind: int) -> float:
    """bin centre exactly as sum(relv_thresholds[k][v])/2 (bpe.py:1509)."""
    return sum(values[ind]) / 2


BOND_LENGTHS = {"N:CA": 1.46, "CA:C": 1.54, "0C:1N": 1.34}  # nerf.py:17-19, used by std_bonds


def residue_token_dict(sym: int, thr: dict, B: int) -> dict:
    """The centre-valued geo dict of a residue symbol, keys in token_geo insertion
    order then as json.dumps(sort_keys=True) would order them."""
    if sym >= B ** 3:
        tau = sym - B ** 3
        d = {"N:CA": [BOND_LENGTHS["N:CA"]], "CA:C": [BOND_LENGTHS["CA:C"]],
             "tau": [centre(thr["tau"], tau)]}
    else:
        tau, cac1n, psi = sym // (B * B), sym // B % B, sym % B
        d = {"N:CA": [BOND_LENGTHS["N:CA"]], "CA:C": [BOND_LENGTHS["CA:C"]], "0C:1N": [BOND_LENGTHS["0C:1N"]],
             "tau": [centre(thr["tau"], tau)], "CA:C:1N": [centre(thr["CA:C:1N"], cac1n)],
             "psi": [centre(thr["psi"], psi)]}
    return d
