"""bpe_iter=*.pkl checkpoints (geobpe.refpickle) against the reference's own
pickled BPE object (tests/golden/<name>.pkl.json, made by
tests/golden/make_pickle_golden.py from /root/reference foldingdiff/bpe.py).

The run state comes from the CPU oracle (pinned to the same fixtures), so these
tests need no GPU; tests/test_bpe_api.py writes the same file from the HIP path."""
import io
import json
import math
import os
import pickle
import subprocess
import sys

import numpy as np
import pytest

from conftest import GOLDEN, REPO, load_golden, pickle_golden_names


def _digest(name):
    with open(os.path.join(GOLDEN, name + ".pkl.json")) as f:
        return json.load(f)


def oracle_run(oracle_lib, name, merges):
    meta, corpus, _ = load_golden(name)
    B = meta["bins"]["1"]
    o = oracle_lib.OracleBPE(corpus, B, cover=meta.get("bin_strategy") == "histogram-cover",
                             strategy=meta.get("bin_strategy")).initialize()
    o.bin()
    for _ in range(merges):
        assert o.step() is not None
    s, ids, off = o.segmentation()
    a, b, eoff = o.events()
    thr = {k: [tuple(p) for p in v] for k, v in o.thresholds.items()}
    run = {
        "corpus": corpus, "fnames": [f"synthetic_{i}" for i in range(len(corpus["row_off"]) - 1)],
        "B": B, "bins": {1: B}, "bin_strategy": meta.get("bin_strategy", "histogram"),
        "thresholds": thr, "bin_counts": meta["api"]["bin_counts"], "K0": o.K0, "tokens": o.vocab(),
        "seg_start": s, "seg_id": ids, "seg_off": off, "ev_a": a, "ev_b": b, "ev_off": eoff,
        "step": merges, "times": [0.0] * merges, "args": {"seed": 0},
    }
    return o, run


def _num(x):
    x = float(x)
    return None if math.isnan(x) else x


def _tree(node):
    return None if node is None else [list(node.value), _tree(node.left), _tree(node.right)]


def _globals(data):
    sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
    from make_pickle_golden import pickle_globals
    return pickle_globals(data)


def check_against_digest(obj, d, merge_keys):
    """A built checkpoint object (geobpe.refpickle.build) against the digest of
    the reference's pickled BPE after the same merges."""
    from geobpe import refpickle
    buf = io.BytesIO()
    refpickle.dump(obj, buf)
    data = buf.getvalue()
    assert _globals(data) == d["globals"]
    bpe = refpickle.load(data)
    assert type(bpe).__module__ == "foldingdiff.bpe" and type(bpe).__name__ == "BPE"
    assert {k: type(v).__name__ for k, v in bpe.__dict__.items()} == d["bpe_attrs"]
    assert {k: type(v).__name__ for k, v in bpe.tokenizers[0].__dict__.items()} == d["tok_attrs"]
    for k, v in d["scalars"].items():
        got = getattr(bpe, k)
        assert (got if not (isinstance(got, float) and math.isinf(got)) else None) == v, k
    assert json.loads(json.dumps({str(k): v for k, v in bpe._thresholds.items()})) == d["thresholds"]
    assert {str(k): {t: [int(x) for x in v] for t, v in g.items()} for k, g in bpe._bin_counts.items()} == d["bin_counts"]
    assert {str(k): {t: v.tolist() for t, v in g.items()} for k, g in bpe._bin_centers.items()} == d["bin_centers"]
    assert {str(k): {t: v.tolist() for t, v in g.items()} for k, g in bpe._bin_weights.items()} == d["bin_weights"]
    assert json.loads(json.dumps([[k, v] for k, v in bpe._tokens.items()])) == d["tokens"]
    assert {k: sorted(list(x) for x in v) for k, v in bpe._geo_dict.items()} == {k: v for k, v in d["geo_dict"]}
    assert [list(p) for p in bpe._priority_dict.keys()] == d["priority_order"]
    assert {k: list(v) for k, v in bpe._key_to_priority.items()} == {k: v for k, v in d["key_to_priority"]}
    assert [[k, v] for k, v in bpe._geo_step.items()] == d["geo_step"]
    assert len(bpe.tokenizers) == len(d["tokenizers"])
    for t, td in zip(bpe.tokenizers, d["tokenizers"]):
        df = t._angles_and_dists
        assert list(df.columns) == td["columns"]
        assert [str(x) for x in df.dtypes] == td["dtypes"]
        assert {c: [_num(v) for v in df[c]] for c in df.columns} == td["values"]
        assert [str(x) for x in t._angles_and_dists_orig.dtypes] == td["orig_dtypes"]
        assert [[k, list(v)] for k, v in t._bond_to_token.items()] == td["bond_to_token"]
        assert t.token_pos == td["token_pos"]
        assert [list(x) for x in t.tokens] == td["tokens"]
        assert [[k, _tree(v)] for k, v in t._bond_to_token.tree.nodes.items()] == td["tree_nodes"]
        assert [[k, list(v.value)] for k, v in t._bond_to_token.tree.leaves.items()] == td["tree_leaves"]
        assert t._bond_to_token.parent is t
        for k in ("n", "fname", "bond_labels", "edges", "_idxes", "compute_sec_structs"):
            assert getattr(t, k) == td[k], k
        assert [int(x) for x in t.atom_labels] == td["atom_labels"]
        assert [[k, v] for k, v in t._res_idx_map.items()] == td["_res_idx_map"]
        assert [t._init_n_ca, t._init_ca_c, t._init_bond_angle] == td["_init"]
        assert sorted(k for k, v in t.__dict__.items() if v is None) == td["none_attrs"]
    assert refpickle.merge_keys(bpe) == merge_keys


@pytest.mark.parametrize("name", pickle_golden_names())
def test_checkpoint_matches_reference_pickle(name, oracle_lib):
    from geobpe import refpickle
    d = _digest(name)
    o, run = oracle_run(oracle_lib, name, d["merges"])
    check_against_digest(refpickle.build(run), d, [k for k, _ in o.merges])


def test_reader_rejects_unlisted_globals():
    from geobpe import refpickle

    class Evil:
        def __reduce__(self):
            return (os.system, ("true",))
    with pytest.raises(pickle.UnpicklingError):
        refpickle.load(pickle.dumps(Evil()))


def test_reader_runs_no_code_nested_in_storage_bytes(tmp_path):
    """torch.storage._load_from_bytes unpickles its argument with weights_only=False;
    the reader must not hand a nested payload to it."""
    from geobpe import refpickle
    marker = tmp_path / "ran"

    class Evil:
        def __reduce__(self):
            return (os.system, (f"touch {marker}",))

    class Nest:
        def __reduce__(self):
            import torch.storage
            return (torch.storage._load_from_bytes, (pickle.dumps(Evil()),))
    with pytest.raises(Exception):
        refpickle.load(pickle.dumps(Nest()))
    assert not marker.exists(), "a payload nested in _load_from_bytes ran"


def test_save_is_atomic_and_complete(tmp_path, oracle_lib):
    from geobpe import refpickle
    _, run = oracle_run(oracle_lib, "g25x1-12_b3_short", 10)
    p = str(tmp_path / "bpe_iter=10.pkl")
    refpickle.save(run, p)
    assert refpickle.is_complete(p) and not os.path.exists(p + ".tmp")
    with open(p, "rb") as f:
        data = f.read()
    with open(p + ".part", "wb") as f:
        f.write(data[: len(data) // 2])
    assert not refpickle.is_complete(p + ".part")
    assert "foldingdiff" not in sys.modules  # dump's stub modules are gone again


REF_CHECK = r'''
import sys, json, pickle
sys.path.insert(0, sys.argv[1]); sys.path.insert(0, sys.argv[2])
import make_golden as MG
MG._stub_optional_deps()
sys.path.insert(0, "/root/reference")
import foldingdiff.bpe as B
B.BPE.visualize = lambda self, key, path: None
bpe = pickle.load(open(sys.argv[3], "rb"))
out = {"ids": [bpe.quantize(t.tokenize()) for t in bpe.tokenizers], "vocab_size": bpe.vocab_size}
(_, negc, key), _ = bpe._priority_dict.peekitem(0)
bpe.step()
out["next"] = [key, -negc]
out["seg"] = [[[s // 3, v[1]] for s, v in t.bond_to_token.items()] for t in bpe.tokenizers]
print(json.dumps(out))
'''


@pytest.mark.skipif(not os.path.isdir("/root/reference/foldingdiff"), reason="reference not present (GPU box)")
@pytest.mark.parametrize("name", pickle_golden_names())
def test_reference_code_loads_and_resumes_checkpoint(name, tmp_path, oracle_lib):
    """The reference itself unpickles the checkpoint, encodes every chain with
    quantize(t.tokenize()) (bin/train.py:128-131) and resumes training with
    step() (bin/encode.py:398): ids, vocab size and the next merge equal the oracle's."""
    from geobpe import refpickle
    d = _digest(name)
    o, run = oracle_run(oracle_lib, name, d["merges"])
    p = str(tmp_path / f"bpe_iter={d['merges']}.pkl")
    refpickle.save(run, p)
    env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1", MPLBACKEND="Agg", SLURM_CPUS_PER_TASK="0")
    r = subprocess.run([sys.executable, "-W", "ignore", "-c", REF_CHECK, os.path.join(REPO, "pt-bpe_amd"),
                        os.path.join(REPO, "tests", "golden"), p], env=env, capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    e, eoff = o.encode()
    assert out["ids"] == [e[eoff[i]:eoff[i + 1]].tolist() for i in range(len(eoff) - 1)]
    assert out["vocab_size"] == o.vocab_size
    o.step()
    assert out["next"] == list(o.merges[-1])
    s, ids, off = o.segmentation()
    assert out["seg"] == [[[int(s[j]), int(ids[j])] for j in range(off[i], off[i + 1])] for i in range(len(off) - 1)]
