"""Golden digest of the reference's ``bpe_iter=*.pkl`` checkpoint object.

Runs the REFERENCE GeoBPE (scoped mode) in the build container on the corpus of
an existing fixture (``<name>.npz``), exactly as ``bin/encode.py`` would before
``pickle.dump(bpe, ...)`` (bin/encode.py:427), pickles the object, and records
a JSON digest of what a consumer of that pickle sees:

  globals       every (module, name) the pickle stream imports
  bpe / tok     attribute names and types of BPE.__dict__ / Tokenizer.__dict__
  state         _thresholds, _bin_counts, _bin_centers, _bin_weights, _tokens,
                _geo_dict, _priority_dict order, _key_to_priority, _geo_step,
                scalar attributes
  tokenizers    per chain: the _angles_and_dists frame (columns, dtypes,
                values), bond_to_token, token_pos, tokens, the merge tree
                (nodes / leaves) and the fixed attributes

The digest is data (inputs come from the fixture, outputs from the reference);
``tests/test_refpickle.py`` checks ``geobpe.refpickle`` against it.
Run only here (``/root/reference`` does not exist on the GPU box):

    python tests/golden/make_pickle_golden.py [name ...]
"""
from __future__ import annotations

import json
import math
import os
import pickle
import pickletools
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "pt-bpe_amd"))
sys.path.insert(0, HERE)

# fixture name -> merges to run before the checkpoint
PICKLE_FIXTURES = {"g40x50_b5": 30, "g25x1-12_b3_short": 25}


def _num(x):
    x = float(x)
    return None if math.isnan(x) else x


def pickle_globals(data: bytes):
    """Every (module, name) the stream imports, read by an Unpickler whose
    find_class records the name and hands back an inert stand-in."""
    import io

    seen = set()

    class _Inert(dict):
        def __new__(cls, *a, **k):
            return dict.__new__(cls)

        def __init__(self, *a, **k):
            pass

        def __setstate__(self, state):
            pass

        def __call__(self, *a, **k):
            return _Inert()

        def append(self, x):
            pass

        def extend(self, x):
            pass

        def add(self, x):
            pass

    class _Rec(pickle.Unpickler):
        def find_class(self, module, name):
            seen.add((module, name))
            return type(name, (_Inert,), {})

    _Rec(io.BytesIO(data)).load()
    return sorted(list(x) for x in seen)


def tree_digest(node):
    if node is None:
        return None
    return [list(node.value), tree_digest(node.left), tree_digest(node.right)]


def run_one(name: str) -> None:
    import numpy as np
    import make_golden as MG
    from geobpe import synth

    MG._stub_optional_deps()
    sys.path.insert(0, "/root/reference")
    import foldingdiff.bpe as B
    from foldingdiff.tokenizer import Tokenizer

    B.BPE.visualize = lambda self, key, path: None
    meta = json.load(open(os.path.join(HERE, f"{name}.json")))
    arrs = np.load(os.path.join(HERE, f"{name}.npz"))
    corpus = {k: arrs[k] for k in list(synth.COLUMNS) + ["row_off"]}
    structs = []
    for i, row in enumerate(synth.corpus_rows(corpus)):
        s = Tokenizer.init_structure(len(row["phi"]))
        for c in synth.COLUMNS:
            s["angles"][c] = row[c].astype(np.float64)
        s["fname"] = f"synthetic_{i}"
        structs.append(s)
    bpe = B.BPE(structs, bins={1: meta["bins"]["1"]}, bin_strategy=meta["bin_strategy"],
                save_dir=tempfile.mkdtemp(prefix="geobpe_pkl_"), rmsd_partition_min_size=float("inf"),
                res_init=True, std_bonds=True, seed=0)
    bpe.initialize()
    bpe.bin()
    merges = PICKLE_FIXTURES[name]
    for _ in range(merges):
        bpe.step()
    data = pickle.dumps(bpe)
    tdig = []
    for t in bpe.tokenizers:
        df = t._angles_and_dists
        tdig.append({
            "columns": list(df.columns),
            "dtypes": [str(x) for x in df.dtypes],
            "values": {c: [_num(v) for v in df[c]] for c in df.columns},
            "orig_dtypes": [str(x) for x in t._angles_and_dists_orig.dtypes],
            "bond_to_token": [[k, list(v)] for k, v in t.bond_to_token.items()],
            "token_pos": list(t.token_pos),
            "tokens": [list(x) for x in t.tokens],
            "tree_nodes": [[k, tree_digest(v)] for k, v in t.bond_to_token.tree.nodes.items()],
            "tree_leaves": [[k, list(v.value)] for k, v in t.bond_to_token.tree.leaves.items()],
            "n": t.n, "fname": t.fname,
            "bond_labels": list(t.bond_labels), "atom_labels": [int(x) for x in t.atom_labels],
            "edges": t.edges, "_idxes": list(t._idxes), "_res_idx_map": [[k, v] for k, v in t._res_idx_map.items()],
            "_init": [t._init_n_ca, t._init_ca_c, t._init_bond_angle],
            "none_attrs": sorted(k for k, v in t.__dict__.items() if v is None),
            "compute_sec_structs": t.compute_sec_structs,
        })
    scalars = {k: v for k, v in bpe.__dict__.items() if isinstance(v, (bool, int, float, str)) and k != "save_dir"}
    dig = {
        "name": name, "merges": merges,
        "globals": pickle_globals(data),
        "bpe_attrs": {k: type(v).__name__ for k, v in bpe.__dict__.items()},
        "tok_attrs": {k: type(v).__name__ for k, v in bpe.tokenizers[0].__dict__.items()},
        "scalars": {k: (None if isinstance(v, float) and math.isinf(v) else v) for k, v in scalars.items()},
        "bins": {str(k): v for k, v in bpe.bins.items()},
        "thresholds": {str(k): v for k, v in bpe._thresholds.items()},
        "bin_counts": {str(k): {t: [int(x) for x in v] for t, v in d.items()} for k, d in bpe._bin_counts.items()},
        "bin_centers": {str(k): {t: v.tolist() for t, v in d.items()} for k, d in bpe._bin_centers.items()},
        "bin_weights": {str(k): {t: v.tolist() for t, v in d.items()} for k, d in bpe._bin_weights.items()},
        "tokens": [[k, v] for k, v in bpe._tokens.items()],
        "geo_dict": [[k, sorted(list(x) for x in v)] for k, v in bpe._geo_dict.items()],
        "priority_order": [list(p) for p in bpe._priority_dict.keys()],
        "key_to_priority": [[k, list(v)] for k, v in bpe._key_to_priority.items()],
        "geo_step": [[k, v] for k, v in bpe._geo_step.items()],
        "times_len": len(bpe._times), "ious": bpe._ious, "sphere_keys": bpe._sphere_keys,
        "tokenizers": tdig,
        "generator": "tests/golden/make_pickle_golden.py (reference: /root/reference foldingdiff/bpe.py)",
    }
    with open(os.path.join(HERE, f"{name}.pkl.json"), "w") as f:
        json.dump(dig, f)
    print(f"{name}: {len(data)} pickle bytes, {len(dig['globals'])} globals", flush=True)


def main(argv):
    if len(argv) >= 2 and argv[0] == "--one":
        run_one(argv[1])
        return
    env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1", MPLBACKEND="Agg", SLURM_CPUS_PER_TASK="0")
    for name in argv or list(PICKLE_FIXTURES):
        r = subprocess.run([sys.executable, "-W", "ignore", __file__, "--one", name], env=env, check=True,
                           stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, text=True)
        print(r.stdout.strip().splitlines()[-1], flush=True)


if __name__ == "__main__":
    main(sys.argv[1:])
