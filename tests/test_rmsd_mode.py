"""RMSD-partitioned mode against the reference's own outputs.

Fixtures: tests/golden/rm_*.json|npz, made by tests/golden/make_rmsd_mode_golden.py running
foldingdiff.bpe.BPE with a finite rmsd_partition_min_size (p = 0, 2, 3 with and without
rmsd_super_res, and p = 4, which the reference cannot step).  Compared exactly: the
residue partition (token ids, medoid geometries, every chain's geometry after
initialize()), the bin() priorities, every merge popped (including the recurring-key
repeats inside one step() call), _tokens, _sphere_dict keys, segmentation, every chain's final
geometry, quantize() (or the exception the reference raised) and vocab_size.

The GPU tests run the product path (device NeRF / RMSD batches, device thresholds).  The
CPU test runs the same host bookkeeping with the oracle's numpy NeRF / Kabsch standing in
for the device batches (oracle/rmsd.py, oracle/prologue.py: test infrastructure).
"""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN

COLS = ["0C:1N", "N:CA", "CA:C", "phi", "psi", "omega", "tau", "CA:C:1N", "C:1N:1CA"]
NAMES = sorted(f[:-5] for f in os.listdir(GOLDEN) if f.startswith("rm_") and f.endswith(".json"))


def _load(name):
    with open(os.path.join(GOLDEN, name + ".json")) as f:
        meta = json.load(f)
    with np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False) as z:
        arrs = {k: z[k] for k in z.files}
    corpus = {k: arrs[k] for k in COLS + ["row_off"]}
    return meta, corpus, arrs


def _geometry_equal(bpe, arrs, tag):
    g = bpe.geometry()
    for c in COLS:
        a, b = g[c], arrs[f"{tag}_{c}"]
        assert a.shape == b.shape and np.array_equal(a, b, equal_nan=True), f"{tag} geometry {c}"
    init = np.array([ch.init for ch in bpe._chains])
    assert np.array_equal(init, arrs[f"{tag}_init"]), f"{tag} init triples"


def _segmentation(bpe):
    return [[[s, list(v[1]) if isinstance(v[1], tuple) else v[1], v[2]] for s, v in t.bond_to_token.items()]
            for t in bpe.tokenizers]


def run_and_compare(name, device=True):
    from geobpe.bpe import BPE
    from geobpe.rmsd_bpe import RmsdBPE

    meta, corpus, arrs = _load(name)
    bpe = BPE(corpus, bins={int(k): v for k, v in meta["bins"].items()}, rmsd_partition_min_size=meta["rmsd_partition_min_size"],
              rmsd_super_res=meta["rmsd_super_res"], num_partitions={int(k): v for k, v in meta["num_partitions"].items()},
              max_num_strucs=meta["max_num_strucs"], std_bonds=meta.get("std_bonds", True),
              seed=meta["rng_seed"], **({"res_init": True} | meta.get("extra", {})))
    assert isinstance(bpe, RmsdBPE)
    if "init_tokens" not in meta:  # the reference raised in initialize()
        with pytest.raises(Exception) as ei:
            bpe.initialize()
        assert type(ei.value).__name__ == meta["raised"]["type"]
        return bpe
    popped = []
    inner = bpe._merge

    def recording():
        popped.append(list(bpe._priority[0]))
        return inner()

    bpe._merge = recording
    bpe.initialize()
    assert [[list(k) if isinstance(k, tuple) else k, v] for k, v in bpe._tokens.items()] == meta["init_tokens"]
    assert list(getattr(bpe, "_sphere_dict", {})) == meta["init_sphere_keys"]
    assert _segmentation(bpe) == meta["init_segmentation"]
    _geometry_equal(bpe, arrs, "init")
    bpe.bin()
    assert len(bpe._priority) == meta["bin_keys"]
    assert [list(p) for p in bpe._priority[:20]] == meta["bin_top"]
    raised = None
    for call in meta["calls"]:
        n0 = len(popped)
        bpe.step()
        assert popped[n0:] == call["popped"], f"merge {len(popped)}"
        assert (bpe._step, len(bpe._tokens)) == (call["step"], call["n_tokens"])
    if meta["raised"]:
        with pytest.raises(Exception) as ei:
            bpe.step()
        raised = type(ei.value).__name__
        assert raised == meta["raised"]["type"]
        assert popped[-1:] == meta["raised"]["popped_so_far"]
    assert [[list(k) if isinstance(k, tuple) else k, v] for k, v in bpe._tokens.items()] == meta["tokens"]
    assert list(getattr(bpe, "_sphere_dict", {})) == meta["sphere_keys"]
    assert _segmentation(bpe) == meta["segmentation"]
    _geometry_equal(bpe, arrs, "final")
    q = []
    for t in bpe.tokenizers:
        try:
            q.append(bpe.quantize(t))
        except ValueError as e:
            q.append({"raised": type(e).__name__})
    assert q == meta["quantize"]
    assert bpe.vocab_size == meta["vocab_size"]
    if "final_top" in meta:
        assert [list(p) for p in bpe._priority[:20]] == meta["final_top"]
    for i, want in enumerate(meta.get("induce", [])):  # BPE.tokenize of held-out / training chains
        ro = arrs["new_row_off"]
        struct = {"angles": {c: arrs[f"new_{c}"][ro[i]:ro[i + 1]] for c in COLS}, "fname": f"new_{i}"}
        if "raised" in want:
            with pytest.raises(Exception) as ei:
                bpe.tokenize(struct)
            assert type(ei.value).__name__ == want["raised"]
            continue
        t, metrics = bpe.tokenize(struct)
        got = [[s0, list(v[1]) if isinstance(v[1], tuple) else v[1], v[2]] for s0, v in t.bond_to_token.items()]
        assert got == want["segmentation"], f"induce {i}"
        assert metrics["L"] == want["L"], f"induce {i}"
        for c in COLS:
            assert np.array_equal(np.asarray(t._c.cur[c]), arrs[f"new{i}_{c}"], equal_nan=True), f"induce {i} {c}"
        assert np.array_equal(np.array(t._c.init), arrs[f"new{i}_init"])
    return bpe


@pytest.fixture
def host_geometry(monkeypatch):
    """The oracle's numpy NeRF / Kabsch / thresholds in place of the device batches."""
    import oracle.prologue as prologue
    import oracle.rmsd as orm
    from geobpe import rmsd, rmsd_bpe

    monkeypatch.setattr(rmsd, "geo_coords", lambda geos, device=0: [orm.nerf(g) for g in geos])
    monkeypatch.setattr(rmsd, "nerf_packed", lambda off, packed, device=0: orm.nerf_packed(off, packed))
    monkeypatch.setattr(rmsd, "nerf_atoms", lambda off, packed, device=0: orm.nerf_atoms(off, packed))
    monkeypatch.setattr(rmsd, "rmsd_matrix", lambda S, device=0: orm.rmsd_matrix(S))
    monkeypatch.setattr(rmsd, "rmsd_cross", lambda A, B, device=0: np.array([[orm.rmsd(a, b) for b in B] for a in A]))
    monkeypatch.setattr(rmsd_bpe.RmsdBPE, "_grid_thresholds",
                        lambda self: {s: prologue.thresholds(self._corpus, b) for s, b in self.bins.items()})


@pytest.mark.parametrize("name", NAMES)
def test_rmsd_mode_host_logic_matches_reference(name, host_geometry):
    run_and_compare(name)


def test_rmsd_mode_dispatch_and_scope():
    from geobpe.bpe import BPE
    from geobpe.rmsd_bpe import RmsdBPE
    _, corpus, _ = _load(NAMES[0])
    assert isinstance(BPE(corpus, bins={1: 5}, res_init=True), RmsdBPE)  # the reference's default p = 4
    with pytest.raises(NotImplementedError):
        BPE(corpus, bins={1: 5}, res_init=True, rmsd_partition_min_size=3, compute_sec_structs=True)
    assert not isinstance(BPE.__new__(BPE, corpus, bins={1: 5}, res_init=True,
                                      rmsd_partition_min_size=float("inf")), RmsdBPE)
    # bond-level init (res_init=False, bpe.py:397-420) runs in the host mirror at any p; with
    # free bonds or glue optimisation it is not built
    assert isinstance(BPE(corpus, bins={1: 5}, res_init=False, rmsd_partition_min_size=float("inf")), RmsdBPE)
    for kw in (dict(std_bonds=False), dict(glue_opt=True)):
        with pytest.raises(NotImplementedError):
            BPE(corpus, bins={1: 5}, res_init=False, rmsd_partition_min_size=3, **kw)


@pytest.mark.gpu
@pytest.mark.parametrize("name", NAMES)
def test_rmsd_mode_device_matches_reference(name):
    bpe = run_and_compare(name)
    meta = _load(name)[0]
    if meta["rmsd_partition_min_size"] <= 3 and "init_tokens" in meta and meta.get("extra", {}).get("res_init", True):
        assert bpe.assign_calls > 0  # the device RMSD batches ran (bond init: its first partitioned
        #                              merge raises before any, as the reference's does)


REF_RESUME = r'''
import sys, json, pickle, tempfile
import numpy as np
sys.path.insert(0, sys.argv[1]); sys.path.insert(0, sys.argv[2])
import make_golden as MG
MG._stub_optional_deps()
sys.path.insert(0, "/root/reference")
import foldingdiff.bpe as B
from foldingdiff.tokenizer import Tokenizer
from geobpe import synth
B.BPE.visualize = lambda self, key, path: None
Tokenizer.visualize_bonds = lambda self, *a, **k: None
popped = []
inner = B.BPE.step
def rec(self):
    top = self._priority_dict.peekitem(0)[0]
    popped.append([bool(top[0]), int(top[1]), top[2]])
    return inner(self)
B.BPE.step = rec
def tid(v):
    return [int(x) for x in v] if isinstance(v, tuple) else int(v)
def resume(bpe, n):
    calls = []
    for _ in range(n):
        n0 = len(popped)
        bpe.step()
        calls.append({"popped": popped[n0:], "step": bpe._step, "n_tokens": len(bpe._tokens)})
    return {"calls": calls,
            "segmentation": [[[int(s), tid(v[1]), int(v[2])] for s, v in t.bond_to_token.items()] for t in bpe.tokenizers],
            "quantize": [quant(bpe, t) for t in bpe.tokenizers], "vocab_size": bpe.vocab_size}
def quant(bpe, t):
    try:
        return [int(x) for x in bpe.quantize(t)]
    except ValueError as e:  # (a NaN or out-of-range angle between tokens: recorded, as the fixtures do)
        return {"raised": type(e).__name__}
name, k, rest = sys.argv[4], int(sys.argv[5]), int(sys.argv[6])
m = json.load(open(f"{sys.argv[2]}/{name}.json"))
z = np.load(f"{sys.argv[2]}/{name}.npz")
corpus = {c: z[c] for c in synth.COLUMNS + ["row_off"]}
structs = []
for i, row in enumerate(synth.corpus_rows(corpus)):
    s = Tokenizer.init_structure(len(row["phi"]))
    for c in synth.COLUMNS:
        s["angles"][c] = row[c].astype(np.float64)
    s["fname"] = f"synthetic_{i}"
    structs.append(s)
ref = B.BPE(structs, bins={int(a): b for a, b in m["bins"].items()}, save_dir=tempfile.mkdtemp(),
            rmsd_partition_min_size=m["rmsd_partition_min_size"], rmsd_super_res=m["rmsd_super_res"],
            num_partitions={int(a): b for a, b in m["num_partitions"].items()}, max_num_strucs=m["max_num_strucs"],
            std_bonds=m.get("std_bonds", True), seed=0, **({"res_init": True} | m.get("extra", {})))
ref.initialize()
ref.bin()
for _ in range(k):
    ref.step()
own = resume(pickle.loads(pickle.dumps(ref)), rest)   # the reference resuming its own checkpoint
ours = resume(pickle.load(open(sys.argv[3], "rb")), rest)
print("JSON" + json.dumps({"own": own, "ours": ours}))
'''


@pytest.mark.skipif(not os.path.isdir("/root/reference/foldingdiff"), reason="reference not present (GPU box)")
@pytest.mark.parametrize("name", ["rm_p0", "rm_p0_multigrid", "rm_p0_super", "rm_pinf_bondinit"])
def test_reference_resumes_rmsd_mode_checkpoint(name, host_geometry, tmp_path):
    """bpe_iter=*.pkl of the RMSD mode: the reference unpickles this build's checkpoint
    taken after 10 step() calls and keeps training.  Its merges, segmentation, quantize ids
    and vocab size equal those of the reference resuming its OWN checkpoint of the same
    point.  (A pickle round trip rebuilds every _geo_dict set, and the order a rebuilt set
    iterates in is what k-medoids sees, bpe.py:1744: with rmsd_super_res or multi-grid
    keys the resumed run can leave the uninterrupted one -- the reference's own resume
    does too.  Where every occurrence of a key is congruent, rm_p0, it also equals the
    uninterrupted run.)"""
    import subprocess
    import sys
    from conftest import REPO
    from geobpe.bpe import BPE
    meta, corpus, _ = _load(name)
    bpe = BPE(corpus, bins={int(k): v for k, v in meta["bins"].items()},
              rmsd_partition_min_size=meta["rmsd_partition_min_size"], rmsd_super_res=meta["rmsd_super_res"],
              num_partitions={int(k): v for k, v in meta["num_partitions"].items()},
              max_num_strucs=meta["max_num_strucs"], std_bonds=meta.get("std_bonds", True),
              seed=meta["rng_seed"], **({"res_init": True} | meta.get("extra", {})))
    bpe.initialize()
    bpe.bin()
    k = 10
    for _ in range(k):
        bpe.step()
    p = str(tmp_path / f"bpe_iter={k}.pkl")
    bpe.save_checkpoint(p)
    env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1", MPLBACKEND="Agg", SLURM_CPUS_PER_TASK="2",
               PYTHONBREAKPOINT="0")
    rest = len(meta["calls"]) - k
    r = subprocess.run([sys.executable, "-W", "ignore", "-c", REF_RESUME, os.path.join(REPO, "pt-bpe_amd"),
                        os.path.join(REPO, "tests", "golden"), p, name, str(k), str(rest)], env=env,
                       capture_output=True, text=True, timeout=1200)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("JSON")][-1][4:])
    assert out["ours"] == out["own"]
    assert out["ours"]["calls"] == meta["calls"][k:]
    if name == "rm_p0":
        assert out["ours"]["segmentation"] == meta["segmentation"]
        assert out["ours"]["quantize"] == meta["quantize"]


@pytest.mark.parametrize("name", ["rm_p0_super", "rm_p2_super_b3"])
def test_induce_cli_rmsd_mode(name, host_geometry, tmp_path):
    _induce_cli(name, tmp_path)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["rm_p0_super", "rm_p2_super_b3", "rm_pdb72_readme"])
def test_induce_cli_rmsd_mode_device(name, tmp_path):
    _induce_cli(name, tmp_path)


def _induce_cli(name, tmp_path):
    """bin/induce.py on a checkpoint of the RMSD mode: the trained run (this build) is
    saved as bpe_iter=*.pkl, the CLI tokenizes the fixture's held-out chains (those the
    reference tokenized without error), and the output pickle's tokenizers carry the
    reference's segmentation of each."""
    import importlib.util
    from conftest import REPO
    from geobpe import refpickle, synth
    from geobpe.bpe import BPE
    meta, corpus, arrs = _load(name)
    bpe = BPE(corpus, bins={int(k): v for k, v in meta["bins"].items()},
              rmsd_partition_min_size=meta["rmsd_partition_min_size"], rmsd_super_res=meta["rmsd_super_res"],
              num_partitions={int(k): v for k, v in meta["num_partitions"].items()},
              max_num_strucs=meta["max_num_strucs"], res_init=True, std_bonds=meta.get("std_bonds", True),
              seed=meta["rng_seed"])
    bpe.initialize()
    bpe.bin()
    for _ in meta["calls"]:
        bpe.step()
    src = tmp_path / "train" / f"bpe_iter={len(meta['calls'])}.pkl"
    src.parent.mkdir()
    bpe.save_checkpoint(str(src))
    ok = [i for i, w in enumerate(meta["induce"]) if "raised" not in w]
    ro = arrs["new_row_off"]
    rows = [{c: arrs[f"new_{c}"][ro[i]:ro[i + 1]] for c in COLS} for i in ok]
    new = {c: np.concatenate([r[c] for r in rows]) for c in COLS}
    new["row_off"] = np.concatenate([[0], np.cumsum([len(r["phi"]) for r in rows])]).astype(np.int64)
    synth.save_corpus(str(tmp_path / "new.npz"), new)
    spec = importlib.util.spec_from_file_location("geobpe_induce_cli", os.path.join(REPO, "pt-bpe_amd", "bin", "induce.py"))
    cli = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(cli)
    out = tmp_path / "out"
    assert cli.main(["--src-pkl", str(src), "--data-dir", str(tmp_path / "new.npz"), "--save-dir", str(out),
                     "--log-dir", str(tmp_path / "logs")]) == 0
    obj = refpickle.load(str(out / src.name))
    assert len(obj.tokenizers) == len(ok)
    for t, i in zip(obj.tokenizers, ok):
        got = [[s0, list(v[1]) if isinstance(v[1], tuple) else v[1], v[2]] for s0, v in t._bond_to_token.items()]
        assert got == meta["induce"][i]["segmentation"]
    assert (out / "utility.json").exists()


@pytest.mark.parametrize("name", ["rm_p0_multigrid", "rm_p3_super_multigrid", "rm_p2_freebonds_multigrid"])
def test_pair_key_c_matches_python(name, host_geometry):
    """csrc/rmsdkey.c (the pair key the host bookkeeping derives twice per merged occurrence)
    against its Python restatement RmsdBPE._pair_key_py, on every adjacent token pair of every
    chain after initialize(), after 6 merges and after 12 (partitioned and plain tokens, pt1 /
    pt2 mixes, several grids); then a value outside the bins raises the same ValueError."""
    from geobpe import rmsd_bpe
    from geobpe.bpe import BPE
    assert rmsd_bpe._KEYC is not None, "pt-bpe_amd/geobpe/_rmsdkey.so is not built (geobpe/build.py)"
    meta, corpus, arrs = _load(name)
    if "init_tokens" not in meta:
        pytest.skip("the reference raised in initialize()")
    bpe = BPE(corpus, bins={int(k): v for k, v in meta["bins"].items()}, rmsd_partition_min_size=meta["rmsd_partition_min_size"],
              rmsd_super_res=meta["rmsd_super_res"], num_partitions={int(k): v for k, v in meta["num_partitions"].items()},
              max_num_strucs=meta["max_num_strucs"], res_init=True, std_bonds=meta.get("std_bonds", True),
              seed=meta["rng_seed"])
    bpe.initialize()
    bpe.bin()

    def both(ci, i1, l1, l2):
        def one(py):
            bpe._py_keys = py
            try:
                return bpe._pair_key(ci, i1, l1, l2)
            except ValueError as e:
                return ("ValueError", str(e))
            finally:
                bpe._py_keys = False
        return one(False), one(True)

    n = 0
    for steps in (0, 6, 6):
        for _ in range(steps):
            bpe.step()
        for ci, c in enumerate(bpe._chains):
            toks = c.tokens()
            for (i1, _, l1), (_, _, l2) in zip(toks, toks[1:]):
                kc, kp = both(ci, i1, l1, l2)
                assert kc == kp, (ci, i1, l1, l2)
                n += 1
    assert n > 500
    # a value outside every bin: the reference's ValueError, the same message both ways
    c = bpe._chains[0]
    toks = c.tokens()
    (i1, _, l1), (_, _, l2) = toks[0], toks[1]
    for k in ("psi", "tau", "CA:C:1N"):
        c.cur[k] = [v + 40.0 for v in c.cur[k]]
    kc, kp = both(0, i1, l1, l2)
    assert kc == kp


@pytest.mark.parametrize("name", ["rm_p0", "rm_p0_super", "rm_p0_b1_one_partition", "rm_p0_multigrid"])
def test_pair_key_memo_equals_derived_keys(name, host_geometry):
    """rmsdkey.c's pair-key memo (partitioned tokens keep their medoid geometry, so a pair's key
    is a function of the two token ids and the junction's three values): with memo_check on,
    every memo hit is derived again from the geometry and must be the same string; the run
    equals the reference's fixture (run_and_compare) and the memo was actually used."""
    from geobpe import rmsd_bpe
    assert rmsd_bpe._KEYC is not None
    rmsd_bpe._KEYC.memo_check(True)
    try:
        bpe = run_and_compare(name)
        hits = rmsd_bpe._KEYC.memo_check(False)
    finally:
        rmsd_bpe._KEYC.memo_check(False)
    n = rmsd_bpe._KEYC.memo_len(bpe._key_memo)
    assert n > 0 and hits > 0, (n, hits)


def test_pair_key_missing_thresholds_raises_like_python(host_geometry):
    """An item type with no thresholds at the span's length: the C key raises the
    exception the Python restatement (the reference's lookup) raises, type and message."""
    from geobpe import rmsd_bpe
    from geobpe.bpe import BPE
    meta, corpus, arrs = _load("rm_p0")
    bpe = BPE(corpus, bins={int(k): v for k, v in meta["bins"].items()}, rmsd_partition_min_size=0,
              num_partitions={int(k): v for k, v in meta["num_partitions"].items()},
              max_num_strucs=meta["max_num_strucs"], res_init=True, seed=meta["rng_seed"])
    bpe.initialize()
    bpe.bin()
    c = bpe._chains[0]
    (i1, _, l1), (_, _, l2) = c.tokens()[0], c.tokens()[1]
    L = l1 + l2

    class NoOmega(dict):
        def __getitem__(self, k):
            if k == "omega":  # (a junction dihedral: binned in every pair key)
                raise KeyError(k)
            return dict.__getitem__(self, k)

    bpe._thr_by_len[L] = NoOmega(bpe._thresholds[L])
    bpe._key_edges.pop(L, None)
    got = []
    for py in (False, True):
        bpe._py_keys = py
        with pytest.raises(KeyError) as e:
            bpe._pair_key(0, i1, l1, l2)
        got.append((type(e.value), e.value.args))
    bpe._py_keys = False
    assert rmsd_bpe._KEYC is not None and got[0] == got[1]


def test_key_float_repr_matches_python():
    """csrc/frepr.cpp (std::to_chars' shortest digits laid out as float.__repr__ does) against
    Python's repr on 200 000 doubles: random bit patterns (subnormals, huge exponents), scaled
    uniforms across 40 decades, three-decimal values, and the edges of the fixed / exponent
    layouts."""
    from geobpe import rmsd_bpe
    assert rmsd_bpe._KEYC is not None, "pt-bpe_amd/geobpe/_rmsdkey.so is not built (geobpe/build.py)"
    rng = np.random.default_rng(17)
    bits = rng.integers(0, 2 ** 63, size=80_000, dtype=np.int64).view(np.float64)
    bits = bits[np.isfinite(bits)]
    sc = rng.random(80_000) * 10.0 ** rng.integers(-20, 20, size=80_000)
    dec = rng.integers(-100_000, 100_000, size=40_000) / 1000.0
    edge = [0.0, -0.0, 1e-4, 9.999999999999999e-05, 1e-5, 1e16, 9999999999999998.0, 1234567890123456.0,
            12345678901234567.0, 0.1, 2 / 3, 1.5e300, 5e-324, 2.2250738585072014e-308, 6.283185307179586]
    vals = [float(v) for v in np.concatenate([bits, sc, dec, -sc])] + edge
    got = rmsd_bpe._KEYC.reprs(vals)
    bad = [(v, g) for v, g in zip(vals, got) if g != repr(v)]
    assert not bad, bad[:5]


def test_set_geo_c_matches_python():
    """csrc/rmsdkey.c setgeo (Tokenizer.set_token_geo into the chain's column lists) against the
    Python version on random spans of fixture chains, and the fallback on values that do not
    fit (the Python version then raises as the reference does)."""
    import copy
    from geobpe import rmsd_bpe
    assert rmsd_bpe._KEYC is not None, "pt-bpe_amd/geobpe/_rmsdkey.so is not built (geobpe/build.py)"

    class PyDict(dict):  # (type(vals) is not dict: the Python path)
        pass

    meta, corpus, arrs = _load("rm_p0_multigrid")
    ro = corpus["row_off"]
    rng = np.random.default_rng(5)
    n = 0
    for r in range(min(12, len(ro) - 1)):
        cols = {c: corpus[c][ro[r]:ro[r + 1]] for c in COLS}
        base = rmsd_bpe._Chain(cols, (1.46, 1.52, 1.94))
        for _ in range(40):
            l = int(rng.integers(1, min(12, 3 * base.n - 1) + 1))
            idx = int(rng.integers(0, 3 * base.n - l + 1))
            vals = {k: [v + 0.25 for v in vs] for k, vs in base.geo(idx, l).items()}
            a, b = copy.deepcopy(base), copy.deepcopy(base)
            a.set_geo(idx, l, vals)
            b.set_geo(idx, l, PyDict(vals))
            assert a.cur == b.cur and a.init == b.init, (r, idx, l)
            n += 1
    assert n > 300
    # values that do not fit: too many, too few, an unknown type -- the Python error either way
    c = rmsd_bpe._Chain({k: corpus[k][ro[0]:ro[1]] for k in COLS}, (1.46, 1.52, 1.94))
    good = c.geo(3, 5)
    for bad in ({**good, "N:CA": good["N:CA"] + [1.0]}, {**good, "CA:C": good["CA:C"][:-1]}, {**good, "x": [1.0]}):
        errs = []
        for v in (bad, PyDict(bad)):
            try:
                copy.deepcopy(c).set_geo(3, 5, v)
                errs.append(None)
            except Exception as e:  # noqa: BLE001
                errs.append((type(e), str(e)))
        assert errs[0] == errs[1] and errs[0] is not None


def test_prio_queue_order_matches_sorted_container():
    """rmsd_bpe._PrioQueue (a lazy-deletion heap over _key_to_priority) against the reference's
    sorted container of (not partitioned, -count, key): the same top after every batch of
    priority updates -- the C path (rmsdkey.prio) and the Python path (remove / add) -- the same
    sorted iteration and slices."""
    import heapq

    from sortedcontainers import SortedList
    from geobpe import rmsd_bpe

    rng = np.random.default_rng(5)
    keys = [f'{{"k": [{i}]}}' for i in range(400)]
    k2p = {k: (True, -int(rng.integers(1, 40)), k) for k in keys[:300]}
    ref = SortedList(k2p.values())
    q = rmsd_bpe._PrioQueue(k2p)
    gd = {k: set(range(-p[1])) for k, p in k2p.items()}
    spheres = {}
    for step in range(300):
        diff = {}
        for k in rng.choice(keys, 12, replace=False):
            k = str(k)
            cur = len(gd.get(k, ()))
            d = int(rng.integers(-cur, 6))
            gd[k] = set(range(cur + d))
            diff[k] = diff.get(k, 0) + d
            if rng.random() < 0.05:
                spheres[k] = None
        use_c = rmsd_bpe._KEYC is not None and step % 2 == 0
        if use_c:
            for k in diff:  # (what the C call does, on the reference container)
                pr = next((p for p in ref if p[2] == k), None)
                if pr is not None:
                    ref.remove(pr)
            rmsd_bpe._KEYC.prio(diff, k2p, q.heap, heapq.heappush, gd, spheres)
            for k in diff:
                if k in k2p:
                    ref.add(k2p[k])
        else:
            for k, d in diff.items():
                pr = k2p.pop(k, None)
                if pr is not None:
                    q.remove(pr)
                    ref.remove(pr)
                n = len(gd[k])
                if n:
                    pr = (k not in spheres, -n, k)
                    k2p[k] = pr
                    q.add(pr)
                    ref.add(pr)
                else:
                    gd.pop(k)
        for k in [k for k in list(gd) if not gd[k]]:
            gd.pop(k)
        assert len(q) == len(ref)
        if len(ref):
            assert q[0] == ref[0]
        if step % 50 == 0:
            assert list(q) == list(ref) and q[:7] == list(ref[:7])


def _group_worker(rank, world, port, names, q, device=False, ckdir="."):
    """one rank of a gloo group running the RMSD mode on the whole corpus: on the GPU (device)
    or with the oracle's stand-ins for the device batches (the host_geometry fixture, by hand:
    no pytest here)"""
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(os.path.dirname(here), "pt-bpe_amd"))
    sys.path.insert(0, os.path.dirname(here))
    sys.path.insert(0, here)
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle.prologue as prologue
        import oracle.rmsd as orm
        from geobpe import rmsd, rmsd_bpe
        from geobpe.bpe import BPE
        if not device:
            rmsd.nerf_atoms = lambda off, packed, device=0: orm.nerf_atoms(off, packed)
            rmsd.nerf_packed = lambda off, packed, device=0: orm.nerf_packed(off, packed)
            rmsd.geo_coords = lambda geos, device=0: [orm.nerf(g) for g in geos]
            rmsd.rmsd_matrix = lambda S, device=0: orm.rmsd_matrix(S)
            rmsd.rmsd_cross = lambda A, B, device=0: np.array([[orm.rmsd(a, b) for b in B] for a in A])
            rmsd_bpe.RmsdBPE._grid_thresholds = lambda self: {s: prologue.thresholds(self._corpus, b)
                                                              for s, b in self.bins.items()}
        for name in names:
            meta, corpus, _ = _load(name)
            bpe = BPE(corpus, bins={int(k): v for k, v in meta["bins"].items()},
                      rmsd_partition_min_size=meta["rmsd_partition_min_size"], rmsd_super_res=meta["rmsd_super_res"],
                      num_partitions={int(k): v for k, v in meta["num_partitions"].items()},
                      max_num_strucs=meta["max_num_strucs"], std_bonds=meta.get("std_bonds", True),
                      seed=meta["rng_seed"], group=True, **({"res_init": True} | meta.get("extra", {})))
            calls = []
            bpe.initialize()
            bpe.bin()
            for _ in meta["calls"]:
                n0 = len(bpe._merge_log)
                bpe.step()
                calls.append([[k, c] for k, c in bpe._merge_log[n0:]])
            want = [[[p[2], -p[1]] for p in c["popped"]] for c in meta["calls"]]
            assert calls == want, f"{name}: merges differ"
            assert _segmentation(bpe) == meta["segmentation"], f"{name}: segmentation"
            assert bpe.assign_calls > 0
        # seed=None (the reference's default): rank 0's seed is broadcast, so every rank draws the
        # same active subsets and medoids; rank 0 alone writes the checkpoint, and no
        # rank returns before it is there
        meta, corpus, _ = _load(names[0])
        bpe = BPE(corpus, bins={int(k): v for k, v in meta["bins"].items()},
                  rmsd_partition_min_size=meta["rmsd_partition_min_size"], rmsd_super_res=meta["rmsd_super_res"],
                  num_partitions={int(k): v for k, v in meta["num_partitions"].items()},
                  max_num_strucs=meta["max_num_strucs"], seed=None, group=True, res_init=True)
        state0 = repr(bpe.rng.bit_generator.state)
        bpe.initialize()
        bpe.bin()
        for _ in range(3):
            bpe.step()
        ck = os.path.join(ckdir, "bpe_iter=3.pkl")
        bpe.save_checkpoint(ck)
        assert os.path.exists(ck), "returned before rank 0's checkpoint"
        q.put((rank, ("ok", state0, [[k, c] for k, c in bpe._merge_log], _segmentation(bpe))))
    except Exception as e:  # pragma: no cover
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


def test_rmsd_mode_process_group_gloo():
    """RmsdBPE(group=...) at world size 2 over gloo: each rank assigns half of every merge's
    occurrences and the halves are all-gathered; both ranks reproduce the reference's merges and
    segmentation (the single-process fixtures)."""
    _group_run(False)


@pytest.mark.gpu
def test_rmsd_mode_process_group_device():
    """The same with the device batches: two ranks on one GPU, gloo for the all-gather."""
    _group_run(True)


def _group_run(device):
    import multiprocessing as mp
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    names = ["rm_p0_super", "rm_p2_super_b3"]
    import tempfile
    with tempfile.TemporaryDirectory() as ckdir:
        ps = [ctx.Process(target=_group_worker, args=(r, 2, port, names, q, device, ckdir)) for r in range(2)]
        for p in ps:
            p.start()
        res = dict(q.get(timeout=600) for _ in ps)
        for p in ps:
            p.join(timeout=60)
    assert all(isinstance(v, tuple) and v[0] == "ok" for v in res.values()), res
    assert res[0][1:] == res[1][1:], "seed=None: the ranks drew differently"


def test_checkpoint_loaded_instance_has_every_init_attribute(host_geometry, tmp_path):
    """RmsdBPE.from_checkpoint skips __init__: every attribute a constructed instance carries
    (its __dict__ and the class defaults) must be on the loaded one too -- round 5's group code
    read an attribute only __init__ set, and a checkpoint-loaded instance failed on the GPU box
    (VERDICT r5 weak 1).  Then the loaded instance tokenizes a chain."""
    from geobpe import refpickle
    from geobpe.bpe import BPE
    from geobpe.rmsd_bpe import RmsdBPE

    meta, corpus, arrs = _load("rm_p0_super")
    bpe = BPE(corpus, bins={int(k): v for k, v in meta["bins"].items()},
              rmsd_partition_min_size=meta["rmsd_partition_min_size"], rmsd_super_res=meta["rmsd_super_res"],
              num_partitions={int(k): v for k, v in meta["num_partitions"].items()},
              max_num_strucs=meta["max_num_strucs"], seed=meta["rng_seed"], res_init=True)
    fresh = set(vars(bpe))
    bpe.initialize()
    bpe.bin()
    bpe.step()
    path = str(tmp_path / "bpe_iter=1.pkl")
    bpe.save_checkpoint(path)
    loaded = RmsdBPE.from_checkpoint(refpickle.load(path))
    missing = sorted(a for a in fresh if not hasattr(loaded, a))
    assert not missing, f"from_checkpoint leaves out {missing}"
    cls_attrs = sorted(a for a in vars(RmsdBPE) if a.startswith("_") and not a.startswith("__")
                       and not isinstance(vars(RmsdBPE)[a], property) and not callable(getattr(RmsdBPE, a))
                       and not hasattr(loaded, a))
    assert not cls_attrs, cls_attrs
    ro = corpus["row_off"]
    t, metrics = loaded.tokenize({"angles": {c: corpus[c][ro[0]:ro[1]] for c in COLS}, "fname": "c0"})
    assert t.bond_to_token and "L" in metrics
