"""``bpe_iter=*.pkl`` checkpoints in the reference's own pickle format.

The reference checkpoints by pickling its ``foldingdiff.bpe.BPE`` object
(bin/encode.py:303,333,427); bin/train.py:114-131, bin/predict.py:842,910,
bin/induce.py:160 and scripts/analyze.py:60-63 load that pickle and call the
reference's methods on it (``tokenizers[i].tokenize()``, ``quantize``,
``vocab_size``, ``dequantize``, ``recover``, ``bond_to_token.tree``).  This
module writes the same object graph from a GeoBPE run of this build, so those
consumers (and the reference's own resume) work on it unchanged:

  BPE.__dict__       the constructor attributes, ``_thresholds`` /
                     ``_bin_counts`` / ``_bin_centers`` / ``_bin_weights``
                     (bpe.py:820-876), ``_tokens``, and the pair index of the
                     current segmentation: ``_geo_dict`` {key: {(chain, start bond
                     of the 2nd token)}}, ``_priority_dict`` SortedDict
                     {(True, -count, key): None}, ``_key_to_priority``,
                     ``_geo_step`` {bin-time key: 0} (bpe.py:1431-1474)
  Tokenizer.__dict__ the angle frame with every value the run uses snapped to its
                     bin centre and the std bond lengths (bpe.py:236-261,
                     714-737), the untouched original frame, ``bond_to_token``
                     as a TokenHierarchy whose BinaryTreeBuilder holds the merge
                     tree (data_structures.py:16-60, 200-226), ``token_pos``,
                     ``tokens`` (the initial tokens: bpe.py:1955-1965 never
                     updates them) and the fixed attributes (tokenizer.py:24-61)

Pickle GLOBALs are the reference's (``foldingdiff.bpe BPE``, ...): the classes
below carry those module / qualified names and are bound in ``sys.modules`` only
while ``dump`` runs (or the real classes are used if the reference is imported).
Differences from a reference-written pickle, all outside what the consumers read:
dict insertion order of ``_geo_dict`` / ``_key_to_priority`` (first occurrence
in the final segmentation instead of creation history), ``_times`` (this run's
per-merge times) and the structure inputs this build does not have (coordinates,
side chains, sequence: None, as for angle-only structures).

``load`` reads a checkpoint (this module's or the reference's) through an
Unpickler that only resolves a whitelist of globals and maps the reference
classes onto plain records; ``merge_keys`` recovers the merge list from it.
"""
from __future__ import annotations

import io
import json
import math
import pickle
import sys
import types
from collections import defaultdict

import numpy as np

from .synth import COLUMNS

# ------------------------------------------------------------------ constants
BOND_TYPES = ["N:CA", "CA:C", "0C:1N"]          # tokenizer.py:19
BOND_LENGTHS = {"N:CA": 1.46, "CA:C": 1.54, "0C:1N": 1.34}   # nerf.py:17-19
ANGLE_KEYS = ["tau", "CA:C:1N", "C:1N:1CA", "psi", "omega", "phi"]  # BOND_ANGLES + DIHEDRAL_ANGLES (bpe.py:830)
FRAME_COLUMNS = ["0C:1N", "N:CA", "CA:C", "phi", "psi", "omega", "tau", "CA:C:1N", "C:1N:1CA"]
GLUE_COLUMNS = ("phi", "omega", "C:1N:1CA")    # float64 in the reference frame, the others object
REF_MODULES = {
    "BPE": "foldingdiff.bpe",
    "Tokenizer": "foldingdiff.tokenizer",
    "TokenHierarchy": "foldingdiff.data_structures",
    "BinaryTreeBuilder": "foldingdiff.data_structures",
    "Node": "foldingdiff.data_structures",
    "ThresholdDict": "foldingdiff.data_structures",
}


# ------------------------------------------------------------------ the reference's classes, as records
class _Record:
    """Attribute record standing in for a reference class (no behaviour)."""

    def __repr__(self):
        return f"<{type(self).__module__}.{type(self).__qualname__} {sorted(self.__dict__)}>"


def _cls(name: str, base=_Record):
    return type(name, (base,), {"__module__": REF_MODULES[name], "__qualname__": name})


BPE = _cls("BPE")
Tokenizer = _cls("Tokenizer")
BinaryTreeBuilder = _cls("BinaryTreeBuilder")


class _Node(_Record):
    def __init__(self, value=None, left=None, right=None):
        self.value = value
        self.left = left
        self.right = right


Node = type("Node", (_Node,), {"__module__": REF_MODULES["Node"], "__qualname__": "Node"})
TokenHierarchy = type("TokenHierarchy", (dict,), {"__module__": REF_MODULES["TokenHierarchy"],
                                                  "__qualname__": "TokenHierarchy"})


class _ThresholdBase(dict):
    """data_structures.py:264-296: int-key floor lookup."""

    def __getitem__(self, key):
        if key in self:
            return super().__getitem__(key)
        if isinstance(key, int):
            ks = [k for k in sorted(k for k in self if isinstance(k, int)) if k <= key]
            if ks:
                return super().__getitem__(ks[-1])
        raise KeyError(key)


ThresholdDict = type("ThresholdDict", (_ThresholdBase,), {"__module__": REF_MODULES["ThresholdDict"],
                                                          "__qualname__": "ThresholdDict"})
_LOCAL = {"BPE": BPE, "Tokenizer": Tokenizer, "TokenHierarchy": TokenHierarchy,
          "BinaryTreeBuilder": BinaryTreeBuilder, "Node": Node, "ThresholdDict": ThresholdDict}


def _real_or_local():
    """The reference classes if the reference is imported in this process, else ours."""
    out = {}
    for name, mod in REF_MODULES.items():
        m = sys.modules.get(mod)
        real = getattr(m, name, None) if m is not None and not getattr(m, "_geobpe_stub", False) else None
        out[name] = real if isinstance(real, type) else _LOCAL[name]
    return out


def _new(cls, attrs: dict):
    o = cls.__new__(cls)
    o.__dict__.update(attrs)
    return o


def _new_dict(cls, items, attrs: dict):
    o = cls.__new__(cls)
    for k, v in items:
        dict.__setitem__(o, k, v)  # not the subclass __setitem__ (TokenHierarchy's records merges)
    o.__dict__.update(attrs)
    return o


# ------------------------------------------------------------------ geometry helpers
def _wrap(v):
    return (v + 2 * np.pi) % (2 * np.pi)


def _get_ind(values, v: float) -> int:
    """BPE.get_ind (bpe.py:1164-1189)."""
    import bisect
    left = [s for s, _ in values]
    i = bisect.bisect_right(left, v) - 1
    if i < 0:
        raise ValueError(f"value {v} is below the first bin range")
    s, e = values[i]
    if (i == len(values) - 1 and v == e) or s <= v < e:
        return i
    raise ValueError(f"value {v} does not fall into any bin")


def _centre(values, i: int) -> float:
    return sum(values[i]) / 2  # bpe.py:1509


def init_bond_angle() -> float:
    from .engine import init_bond_angle as iba
    return iba()


def _fnum(x) -> float:
    return float(x)


def _frame(pd, data: dict, dtypes: dict):
    df = pd.DataFrame({c: pd.Series(data[c], dtype=dtypes[c]) for c in FRAME_COLUMNS})
    return df


def chain_frames(pd, cols: dict, thr: dict):
    """(quantized frame, original frame) of one chain: every value the scoped run
    reads snapped to its bin centre (quant_geo / set_token_geo, bpe.py:236-261,
    381-391, 1500-1526) and the bond lengths of bonds 2..3n-2 set to the standard
    lengths (_set_bond_length_worker, bpe.py:714-737)."""
    n = len(cols["phi"])
    orig = {c: [_fnum(x) for x in cols[c]] for c in FRAME_COLUMNS}
    q = {c: list(v) for c, v in orig.items()}
    for c in BOND_TYPES:
        for r in range(max(n - 1, 0)):
            q[c][r] = BOND_LENGTHS[c]
    for c in ("tau", "CA:C:1N", "psi", "omega", "C:1N:1CA"):
        for r in range(max(n - 1, 0)):
            q[c][r] = _centre(thr[c], _get_ind(thr[c], _wrap(orig[c][r])))
    for r in range(1, n):
        q["phi"][r] = _centre(thr["phi"], _get_ind(thr["phi"], _wrap(orig["phi"][r])))
    qd = {c: (np.float64 if c in GLUE_COLUMNS else object) for c in FRAME_COLUMNS}
    od = {c: object for c in FRAME_COLUMNS}
    return _frame(pd, q, qd), _frame(pd, orig, od)


# ------------------------------------------------------------------ pair keys
def _res_bins(s: int, B: int):
    """(tau, cac1n, psi) of a residue symbol; the last residue of a chain has only tau."""
    if s >= B ** 3:
        return (s - B ** 3, None, None)
    return (s // (B * B), s // B % B, s % B)


def span_key(rsym, gsym, a: int, b: int, last: bool, B: int) -> str:
    """json.dumps(geo, sort_keys=True) of the bin indices of residues a..b
    (BPE.compute_geo_key, bpe.py:1192-1299; BPE.hash_geo, bpe.py:1147-1149)."""
    r = b - a + 1
    lam = 1 if last else 0
    rb = [_res_bins(int(rsym[j]), B) for j in range(a, b + 1)]
    gb = [(int(gsym[j]) // (B * B), int(gsym[j]) // B % B, int(gsym[j]) % B) for j in range(a, b)]
    geo = {
        "0C:1N": [0] * (r - lam), "C:1N:1CA": [g[1] for g in gb], "CA:C": [0] * r,
        "CA:C:1N": [x[1] for x in rb[: r - lam]], "N:CA": [0] * r, "omega": [g[0] for g in gb],
        "phi": [g[2] for g in gb], "psi": [x[2] for x in rb[: r - lam]], "tau": [x[0] for x in rb],
    }
    return json.dumps(geo, sort_keys=True)


def symbols(cols: dict, thr: dict, B: int):
    """Residue / junction symbols of one chain (k_quantize's layout)."""
    n = len(cols["phi"])
    rs = np.zeros(n, np.int64)
    gs = np.full(n, -1, np.int64)
    ind = lambda k, v: _get_ind(thr[k], _wrap(v))  # noqa: E731
    for j in range(n):
        tau = init_bond_angle() if j == 0 else cols["tau"][j - 1]
        tb = ind("tau", tau)
        if j == n - 1:
            rs[j] = B ** 3 + tb
        else:
            rs[j] = tb * B * B + ind("CA:C:1N", cols["CA:C:1N"][j]) * B + ind("psi", cols["psi"][j])
            gs[j] = (ind("omega", cols["omega"][j]) * B * B + ind("C:1N:1CA", cols["C:1N:1CA"][j]) * B
                     + ind("phi", cols["phi"][j + 1]))
    return rs, gs


# ------------------------------------------------------------------ the checkpoint object
def build_tokenizers(run: dict, C=None):
    """Tokenizer records of a run's chains (frames, bond_to_token with the merge
    tree, token_pos, tokens, fixed attributes) and its pair index
    (``_geo_dict`` / ``_geo_step``).  ``run["sym_of_label"]`` fixes the residue
    labels of a trained vocabulary (merge replay); default: first appearance."""
    import pandas as pd

    C = C or _real_or_local()
    corpus = run["corpus"]
    ro = np.asarray(corpus["row_off"], dtype=np.int64)
    B = int(run["B"])
    thr1 = {k: [tuple(map(float, p)) for p in run["thresholds"][k]] for k in ANGLE_KEYS}
    K0 = int(run["K0"])
    nrows = len(ro) - 1
    fnames = run.get("fnames") or [None] * nrows
    seg_start, seg_id, seg_off = (np.asarray(run[k]) for k in ("seg_start", "seg_id", "seg_off"))
    ev_a, ev_b, ev_off = (np.asarray(run[k], dtype=np.int64) for k in ("ev_a", "ev_b", "ev_off"))

    # per chain: symbols, initial tokens, merge tree from the events
    rsyms, gsyms = [], []
    for r in range(nrows):
        cols = {c: np.asarray(corpus[c][ro[r]:ro[r + 1]], dtype=np.float64) for c in COLUMNS}
        rs, gs = symbols(cols, thr1, B)
        rsyms.append(rs)
        gsyms.append(gs)
    if run.get("sym_of_label") is not None:
        label_of_sym = {int(sy): i for i, sy in enumerate(run["sym_of_label"])}
    else:
        allr = np.concatenate(rsyms) if nrows else np.zeros(0, np.int64)
        uniq, first = np.unique(allr, return_index=True)
        label_of_sym = {int(sy): i for i, sy in enumerate(uniq[np.argsort(first, kind="stable")])}
    if len(label_of_sym) != K0:
        raise ValueError(f"{len(label_of_sym)} residue labels, run says K0={K0}")
    chain_of = np.searchsorted(ro, np.arange(int(ro[-1])), side="right") - 1 if nrows else np.zeros(0, np.int64)

    trees = []
    for r in range(nrows):
        n = int(ro[r + 1] - ro[r])
        nodes, leaves = {}, {}
        for j in range(n):
            v = (3 * j, label_of_sym[int(rsyms[r][j])], 3 if j < n - 1 else 2)
            nodes[v[0]] = _new(C["Node"], {"value": v, "left": None, "right": None})
            leaves[v[0]] = _new(C["Node"], {"value": v, "left": None, "right": None})
        trees.append((nodes, leaves))
    for t in range(len(ev_off) - 1):
        nid = K0 + t
        for i in range(int(ev_off[t]), int(ev_off[t + 1])):
            a, b = int(ev_a[i]), int(ev_b[i])
            r = int(chain_of[a])
            nodes = trees[r][0]
            L = nodes.pop(3 * (a - int(ro[r])))
            R = nodes.pop(3 * (b - int(ro[r])))
            v = (L.value[0], nid, L.value[2] + R.value[2])
            nodes[v[0]] = _new(C["Node"], {"value": v, "left": L, "right": R})  # BinaryTreeBuilder.combine

    # pair index of the final segmentation; bin-time keys in first-occurrence order
    geo = defaultdict(set)
    geo_step = {}
    for r in range(nrows):
        n = int(ro[r + 1] - ro[r])
        for j in range(n - 1):
            k = span_key(rsyms[r], gsyms[r], j, j + 1, j + 1 == n - 1, B)
            if k not in geo_step:
                geo_step[k] = 0
        st = [int(x) for x in seg_start[seg_off[r]:seg_off[r + 1]]] + [n]
        for k in range(len(st) - 2):
            key = span_key(rsyms[r], gsyms[r], st[k], st[k + 2] - 1, st[k + 2] == n, B)
            geo[key].add((r, 3 * st[k + 1]))

    tiba = thr1["tau"]
    init_tau = _centre(tiba, _get_ind(tiba, _wrap(init_bond_angle())))
    tokenizers = []
    for r in range(nrows):
        n = int(ro[r + 1] - ro[r])
        cols = {c: np.asarray(corpus[c][ro[r]:ro[r + 1]]) for c in COLUMNS}
        qdf, odf = chain_frames(pd, cols, thr1)
        st = [int(x) for x in seg_start[seg_off[r]:seg_off[r + 1]]]
        ids = [int(x) for x in seg_id[seg_off[r]:seg_off[r + 1]]]
        btt = []
        for k, (s0, v) in enumerate(zip(st, ids)):
            e = st[k + 1] if k + 1 < len(st) else n
            btt.append((3 * s0, (3 * s0, v, 3 * (e - s0) - (1 if e == n else 0))))
        token_pos = []
        for _, (s3, _, nb) in btt:
            token_pos.extend([s3] * nb)
        init_tokens = [(3 * j, label_of_sym[int(rsyms[r][j])], 3) for j in range(n - 1)] + (
            [(3 * n - 3, label_of_sym[int(rsyms[r][n - 1])], 2)] if n else [])
        idxes = sum([[i, i, i] for i in range(1, n + 1)], [])
        tok = _new(C["Tokenizer"], {})
        nodes, leaves = trees[r]
        tree = _new(C["BinaryTreeBuilder"], {"nodes": nodes, "leaves": leaves})
        hier = _new_dict(C["TokenHierarchy"], btt, {"parent": tok, "tree": tree})
        tok.__dict__.update({
            "_angles_and_dists": qdf, "_angles_and_dists_orig": odf, "_coords": None, "beta_coords": None,
            "_idxes": idxes, "_res_idx_map": dict(zip(idxes[0::3], range(0, len(idxes), 3))),
            "_full_coords": None, "compute_sec_structs": False, "_sec": None, "_side_chains": None, "aa": None,
            "fname": fnames[r], "n": n,
            "bond_labels": sum([[0, 1, 2] for _ in range(n - 1)] + [[0, 1]], []),
            "atom_labels": np.tile([0, 1, 2], n), "edges": [[j, j + 1, 0] for j in range(1, 3 * n)],
            "_bond_to_token": hier, "_init_n_ca": BOND_LENGTHS["N:CA"], "_init_ca_c": BOND_LENGTHS["CA:C"],
            "_init_bond_angle": init_tau, "token_pos": token_pos, "tokens": init_tokens,
        })
        tokenizers.append(tok)
    return tokenizers, {"geo": geo, "geo_step": geo_step, "rsyms": rsyms, "thr1": thr1}


def build(run: dict):
    """The reference BPE object graph of a GeoBPE run.

    ``run``: corpus (columns + row_off), fnames, B, bins, bin_strategy,
    thresholds (grid-1 {type: [(start, end)]}), bin_counts ({type: [count]}),
    K0, tokens (BPE._tokens), seg_start / seg_id / seg_off (final segmentation,
    chain-local residue starts), ev_a / ev_b / ev_off (merge events: global
    left / right token start slots, events of merge t in [ev_off[t],
    ev_off[t+1])), step, times, the constructor arguments in ``args``."""
    import pandas as pd
    import torch
    from sortedcontainers import SortedDict

    C = _real_or_local()
    tokenizers, extra = build_tokenizers(run, C)
    geo, geo_step, rsyms = extra["geo"], extra["geo_step"], extra["rsyms"]
    nrows = len(tokenizers)
    thr1 = extra["thr1"]
    prio = SortedDict()
    k2p = {}
    for key, occ in geo.items():
        p = (True, -len(occ), key)
        prio[p] = None
        k2p[key] = p

    # grid-1 state (bpe.py:856-876)
    thresholds = _new_dict(C["ThresholdDict"], [(1, {k: list(v) for k, v in thr1.items()})]
                           + [(bt, [(BOND_LENGTHS[bt], BOND_LENGTHS[bt])]) for bt in BOND_TYPES], {})
    thresholds.__dict__["_int_keys"] = [1]
    counts = {k: [np.int64(c) for c in run["bin_counts"][k]] for k in ANGLE_KEYS}
    bin_counts = _new_dict(C["ThresholdDict"], [(1, counts)], {"_int_keys": [1]})
    centers = _new_dict(C["ThresholdDict"], [(1, {k: torch.tensor(v, dtype=torch.float32).mean(axis=-1)
                                                  for k, v in thr1.items()})], {"_int_keys": [1]})
    weights = _new_dict(C["ThresholdDict"], [(1, {k: torch.tensor(v, dtype=torch.float32) / sum(v)
                                                  for k, v in counts.items()})], {"_int_keys": [1]})

    a = run.get("args", {})
    seed = a.get("seed")
    attrs = {
        "tokenizers": tokenizers,
        "compute_sec_structs": a.get("compute_sec_structs", False),
        "plot_iou_with_sec_structs": a.get("plot_iou_with_sec_structs", False),
        "rmsd_partition_min_size": a.get("rmsd_partition_min_size", float("inf")),
        "rmsd_super_res": a.get("rmsd_super_res", False), "rmsd_only": a.get("rmsd_only", False),
        "glue_opt": a.get("glue_opt", False), "glue_opt_every": a.get("glue_opt_every", 10),
        "glue_opt_prior": a.get("glue_opt_prior", 0.0), "glue_opt_method": a.get("glue_opt_method", "all"),
        "num_partitions": a.get("num_partitions", 3), "max_num_strucs": a.get("max_num_strucs", 500),
        "res_init": True, "std_bonds": True, "bins": dict(run["bins"]), "bin_strategy": run["bin_strategy"],
        "n": nrows, "seed": seed, "rng": np.random.default_rng(seed), "save_dir": a.get("save_dir", "./plots/bpe"),
        "_step": int(run["step"]), "_times": list(run.get("times", [])), "_ious": [],
        "_thresholds": thresholds, "_bin_counts": bin_counts, "_bin_centers": centers, "_bin_weights": weights,
        "_tokens": dict(run["tokens"]), "_geo_dict": geo, "_priority_dict": prio, "_key_to_priority": k2p,
        "_geo_step": geo_step, "_sphere_keys": {},
    }
    return _new(C["BPE"], attrs)


def dump(obj, f) -> None:
    """pickle.dump with the reference's GLOBALs: while it runs, the record
    classes are reachable as foldingdiff.* (unless the reference is imported)."""
    added = []
    try:
        for name, mod in REF_MODULES.items():
            parts = mod.split(".")
            for i in range(1, len(parts) + 1):
                m = ".".join(parts[:i])
                if m not in sys.modules:
                    stub = types.ModuleType(m)
                    stub._geobpe_stub = True
                    stub.__path__ = []
                    sys.modules[m] = stub
                    added.append(m)
            m = sys.modules[mod]
            if getattr(m, "_geobpe_stub", False):
                setattr(m, name, _LOCAL[name])
        pickle.dump(obj, f)
    finally:
        for m in added:
            sys.modules.pop(m, None)


def save(run: dict, path: str) -> None:
    """Write ``path`` atomically (a partial file never looks complete to
    bin/encode.py's is_complete_pickle, encode.py:183-198)."""
    import os
    tmp = path + ".tmp"
    with open(tmp, "wb") as f:
        dump(build(run), f)
    os.replace(tmp, path)


# ------------------------------------------------------------------ reading
_SAFE = {
    ("builtins", "set"), ("builtins", "slice"), ("builtins", "frozenset"), ("collections", "OrderedDict"),
    ("collections", "defaultdict"), ("sortedcontainers.sorteddict", "SortedDict"),
    ("numpy", "dtype"), ("numpy", "ndarray"), ("numpy.core.multiarray", "_reconstruct"),
    ("numpy._core.multiarray", "_reconstruct"), ("numpy.core.multiarray", "scalar"),
    ("numpy._core.multiarray", "scalar"),
    ("numpy.random._pickle", "__generator_ctor"), ("numpy.random._pickle", "__bit_generator_ctor"),
    ("numpy.random._pcg64", "PCG64"), ("numpy.random.bit_generator", "SeedSequence"),
    ("numpy.random.bit_generator", "__pyx_unpickle_SeedSequence"),
    ("pandas._libs.internals", "_unpickle_block"), ("pandas.core.frame", "DataFrame"),
    ("pandas.core.series", "Series"),
    ("pandas.core.indexes.base", "Index"), ("pandas.core.indexes.base", "_new_Index"),
    ("pandas.core.indexes.range", "RangeIndex"), ("pandas.core.internals.managers", "BlockManager"),
    ("pandas.core.internals.managers", "SingleBlockManager"),
    ("torch._utils", "_rebuild_tensor_v2"),
}


def _storage_from_bytes(b):
    """Stand-in for ``torch.storage._load_from_bytes``: torch's own version
    unpickles ``b`` with ``weights_only=False`` (arbitrary code); this one only
    accepts tensor/storage payloads."""
    import torch
    return torch.load(io.BytesIO(b), weights_only=True)


class _Reader(pickle.Unpickler):
    def find_class(self, module, name):
        if REF_MODULES.get(name) == module:
            return _LOCAL[name]
        if (module, name) == ("torch.storage", "_load_from_bytes"):
            return _storage_from_bytes
        if (module, name) in _SAFE:
            if module.startswith("torch"):
                import torch  # noqa: F401
            return super().find_class(module, name)
        raise pickle.UnpicklingError(f"checkpoint global {module}.{name} is not on the reader's whitelist")


def load(path_or_bytes):
    """A checkpoint as records (BPE / Tokenizer / TokenHierarchy / ... with the
    reference attribute names); resolves only whitelisted globals."""
    if isinstance(path_or_bytes, (bytes, bytearray)):
        return _Reader(io.BytesIO(path_or_bytes)).load()
    with open(path_or_bytes, "rb") as f:
        return _Reader(f).load()


def merge_keys(obj) -> list:
    """The merge list (key strings in merge order) of a checkpoint: merged token
    n holds json.loads(key) (bpe.py:1857-1860), so key = json.dumps(_tokens[n],
    sort_keys=True) for n >= K0 (the residue tokens hold bin-centre floats)."""
    toks = obj._tokens
    ids = sorted(toks)
    out = []
    for v in ids:
        d = toks[v]
        vals = [x for lst in d.values() for x in lst]
        if vals and all(isinstance(x, int) for x in vals):
            out.append(json.dumps(d, sort_keys=True))
        elif out:
            raise ValueError(f"token {v}: residue token after merged tokens")
    return out


def is_complete(path: str) -> bool:
    """bin/encode.py:183-198: the pickle bytecode parses to its STOP opcode."""
    import pickletools
    try:
        with open(path, "rb") as f:
            data = f.read()
        for _ in pickletools.genops(data):
            pass
        return True
    except Exception:
        return False


def _is_nan(x):
    return isinstance(x, float) and math.isnan(x)
