"""The drop-in object API (geobpe.bpe.BPE, mirror of foldingdiff.bpe.BPE) against
the reference's own outputs for the same calls (tests/golden/*.json "api")."""
import json

import numpy as np
import pytest

from conftest import golden_names, load_golden


def _bpe(meta, corpus):
    from geobpe.bpe import BPE
    b = BPE(corpus, bins={1: meta["bins"]["1"]}, bin_strategy=meta.get("bin_strategy", "histogram"),
            res_init=True, rmsd_partition_min_size=float("inf"), std_bonds=True, seed=0)
    return b


@pytest.mark.parametrize("kw, exc", [
    (dict(rmsd_partition_min_size=3, glue_opt=True, glue_opt_method="other"), ValueError),
    (dict(rmsd_partition_min_size=2, compute_sec_structs=True), NotImplementedError),
    (dict(glue_opt=True), NotImplementedError),  # glue opt without RMSD partitioning (bpe.py:2027)
    (dict(std_bonds=False), KeyError),  # as the reference's initialize() (free-bonds probe)
    (dict(bin_strategy="quantile"), NotImplementedError),

    (dict(bins={2: 5}), KeyError),
])
def test_out_of_scope_configurations_are_rejected(kw, exc):
    """Scope check happens before any device work (runs without a GPU)."""
    from geobpe.bpe import BPE
    args = dict(bins={1: 5}, res_init=True, rmsd_partition_min_size=float("inf"))
    args.update(kw)
    bins = args.pop("bins")
    with pytest.raises(exc):
        BPE({"row_off": np.zeros(1, dtype=np.int64)}, bins, **args)


def test_reference_probe_of_multigrid_and_free_bonds():
    """Evidence behind the two rejections above (tests/golden/probe_multigrid.py ran
    the reference): with a multi-grid schedule its step() finds a stale neighbour key
    at step 1 (bpe.py:1917-1920) and, with breakpoints disabled, re-selects the same
    key forever without merging; free bonds raise KeyError('N:CA') in initialize()."""
    import os
    from conftest import GOLDEN
    with open(os.path.join(GOLDEN, "multigrid_reference.json")) as f:
        d = json.load(f)
    dbg = d["debugger"]
    assert dbg["stopped"] == "breakpoint at step 1" and dbg["breakpoints"][0]["line"] == 1919
    assert dbg["breakpoints"][0]["differs"]  # stored key != recomputed key
    loop = d["PYTHONBREAKPOINT=0"]["merges"]
    assert len({m["key"] for m in loop[1:]}) == 1  # the same key every step
    assert len({m["live_tokens_before"] for m in loop[1:]}) == 1  # and nothing merges
    assert d["free-bonds"]["raised"] == "KeyError" and d["free-bonds"]["args"] == ["N:CA"]


def test_codebook_utility_matches_definition():
    from geobpe.bpe import get_codebook_utility
    u = get_codebook_utility([0, 0, 1, 3], 4)
    p = np.array([0.5, 0.25, 0, 0.25])
    ent = -np.sum(p * np.log(p + 1e-8))
    assert abs(u["entropy"] - ent) < 1e-6 and u["use_ratio"] == 0.75


def test_threshold_dict_floor_lookup():
    from geobpe.bpe import ThresholdDict
    t = ThresholdDict({1: "a", 5: "b", "N:CA": "c"})
    assert t[1] == "a" and t[4] == "a" and t[5] == "b" and t[99] == "b" and t["N:CA"] == "c"
    with pytest.raises(KeyError):
        t[0]


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["step", "run"])
@pytest.mark.parametrize("name", golden_names())
def test_bpe_object_api_matches_reference(name, mode):
    meta, corpus, arrs = load_golden(name)
    api = meta["api"]
    b = _bpe(meta, corpus)
    b.initialize()
    assert {k: [list(p) for p in v] for k, v in b._thresholds[1].items()} == meta["thresholds"]
    assert b._bin_counts[1] == api["bin_counts"]
    b.bin()
    if mode == "step":
        for _ in range(len(meta["merges"])):
            b.step()
    else:
        assert b.run(len(meta["merges"])) == len(meta["merges"])
    assert b._step == len(meta["merges"])
    assert {str(k): v for k, v in b._tokens.items()} == meta["vocab"]
    assert b.vocab_size == meta["vocab_size"]
    assert {k: b.cum_bin_count(k) for k in meta["cum_bin_count"]} == meta["cum_bin_count"]
    assert b.capacity() == api["capacity"]
    assert abs(b.capacity(tokenizer=True) - api["capacity_tokenizer"]) <= 1e-9 * api["capacity_tokenizer"]
    toks = b.tokenizers
    q = b.quantize(toks)
    flat = np.concatenate([np.asarray(x, dtype=np.int64) for x in q])
    assert np.array_equal(flat, arrs["ids"])
    for i, t in enumerate(toks[:3]):
        assert [list(v) for v in t.bond_to_token.values()] == api["bond_to_token"][i]
        assert t.token_pos == api["token_pos"][i]
        tt = t.tokenize()
        assert [list(x) for x in tt] == api["tokenize"][i]
        assert b.quantize(tt) == b.quantize(t)  # tuple path == tokenizer path
        assert [list(x) for x in b.dequantize(b.quantize(t))] == api["dequantize"][i]
        assert json.loads(json.dumps(b.recover(tt))) == api["recover"][i]
    b.close()


@pytest.mark.gpu
def test_step_past_exhaustion_raises():
    from geobpe import synth
    from geobpe.bpe import BPE
    lengths = synth.make_lengths(6, 1, 6, seed=3)
    b = BPE(synth.make_corpus(lengths, seed=3), {1: 2}, res_init=True,
            rmsd_partition_min_size=float("inf"))
    b.initialize()
    b.bin()
    b.run(10000)
    with pytest.raises(IndexError):
        b.step()
    assert all(len(t.tokens) == 1 for t in b.tokenizers)
    b.close()


def _encode_cli():
    import importlib.util
    import os
    from conftest import REPO
    spec = importlib.util.spec_from_file_location("geobpe_encode_cli", os.path.join(REPO, "pt-bpe_amd", "bin", "encode.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_cli_flags_mirror_reference_parsers():
    cli = _encode_cli()
    a = cli.parse_args(["--save-dir", "x", "--bins", "1-5", "--p-min-size", "inf", "--res-init", "true"])
    assert a.bins == {1: 5} and a.p_min_size == float("inf") and a.res_init is True
    assert cli.str2dict("1-5:10-3") == {1: 5, 10: 3}
    with pytest.raises(Exception):
        cli.str2dict("1-5:")


def test_cli_latest_checkpoint_skips_incomplete(tmp_path, oracle_lib):
    from test_refpickle import oracle_run
    from geobpe import refpickle
    cli = _encode_cli()
    (tmp_path / "bpe_iter=10.json").write_text(json.dumps({"merges": [["k", 1]]}))
    (tmp_path / "bpe_iter=20.json").write_text("{\"merges\": [")  # torn write
    it, path, keys = cli.latest_checkpoint(str(tmp_path))
    assert it == 10 and path.endswith("bpe_iter=10.json") and keys == ["k"]
    o, run = oracle_run(oracle_lib, "g25x1-12_b3_short", 12)
    refpickle.save(run, str(tmp_path / "bpe_iter=12.pkl"))
    data = (tmp_path / "bpe_iter=12.pkl").read_bytes()
    (tmp_path / "bpe_iter=30.pkl").write_bytes(data[: len(data) - 7])  # torn pickle
    it, path, keys = cli.latest_checkpoint(str(tmp_path))
    assert it == 12 and path.endswith("bpe_iter=12.pkl") and keys == [k for k, _ in o.merges]


@pytest.mark.gpu
def test_cli_resume_reproduces_one_shot(tmp_path):
    cli = _encode_cli()
    common = ["--data-dir", "synthetic:300:30:150:5", "--bins", "1-5", "--save-every", "10",
              "--log-dir", str(tmp_path / "logs")]
    one, two = tmp_path / "one", tmp_path / "two"
    assert cli.main(common + ["--save-dir", str(one), "--max-iter", "61"]) == 0
    assert cli.main(common + ["--save-dir", str(two), "--max-iter", "31"]) == 0
    assert cli.main(common + ["--save-dir", str(two), "--max-iter", "61"]) == 0  # resumes at 30
    from geobpe import refpickle
    a = refpickle.merge_keys(refpickle.load(str(one / "bpe_iter=60.pkl")))
    b = refpickle.merge_keys(refpickle.load(str(two / "bpe_iter=60.pkl")))
    assert a == b and len(a) == 61
    sa = json.loads((one / "stats=60.json").read_text())
    assert sa == json.loads((two / "stats=60.json").read_text()) and sa["K"] > 0


@pytest.mark.gpu
def test_cli_rmsd_mode_resume_reproduces_one_shot(tmp_path):
    """bin/encode.py in the RMSD-partitioned mode (--p-min-size 0, --num-p): a run resumed
    at iter 10 ends with the one-shot run's merges and stats, with json checkpoints and with
    bpe_iter=*.pkl (the reference's pickle of this mode: segmentation and geometry too)."""
    from geobpe import refpickle
    cli = _encode_cli()
    for fmt in ("json", "pkl"):
        common = ["--data-dir", "synthetic:40:20:60:9", "--bins", "1-5", "--save-every", "5", "--p-min-size", "0",
                  "--num-p", "2-2:3-3:5-2", "--max-num-strucs", "60", "--rmsd-super-res", "true",
                  "--ckpt-format", fmt, "--log-dir", str(tmp_path / "logs")]
        one, two = tmp_path / f"one_{fmt}", tmp_path / f"two_{fmt}"
        assert cli.main(common + ["--save-dir", str(one), "--max-iter", "21"]) == 0
        assert cli.main(common + ["--save-dir", str(two), "--max-iter", "11"]) == 0
        assert cli.main(common + ["--save-dir", str(two), "--max-iter", "21"]) == 0  # resumes at 10
        if fmt == "json":
            a = json.loads((one / "bpe_iter=20.json").read_text())["merges"]
            b = json.loads((two / "bpe_iter=20.json").read_text())["merges"]
            assert a == b and len(a) >= 20
        else:
            a, b = refpickle.load(str(one / "bpe_iter=20.pkl")), refpickle.load(str(two / "bpe_iter=20.pkl"))
            assert list(a._sphere_dict) == list(b._sphere_dict) and a._step == b._step >= 20
            for ta, tb in zip(a.tokenizers, b.tokenizers):
                assert dict(ta._bond_to_token) == dict(tb._bond_to_token)
                assert ta._angles_and_dists.equals(tb._angles_and_dists)
        assert json.loads((one / "stats=20.json").read_text()) == json.loads((two / "stats=20.json").read_text())


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["g40x50_b5", "g25x1-12_b3_short"])
def test_checkpoint_from_device_matches_reference_pickle(name):
    """BPE.save_checkpoint on the HIP path (device merge-event log for the merge
    tree) against the digest of the reference's own pickled BPE."""
    import os
    from conftest import GOLDEN
    from test_refpickle import check_against_digest
    from geobpe import refpickle
    with open(os.path.join(GOLDEN, name + ".pkl.json")) as f:
        d = json.load(f)
    meta, corpus, _ = load_golden(name)
    from geobpe.bpe import BPE
    b = BPE(corpus, bins={1: meta["bins"]["1"]}, res_init=True, rmsd_partition_min_size=float("inf"), seed=0)
    b._fnames = [f"synthetic_{i}" for i in range(len(corpus["row_off"]) - 1)]
    b.initialize()
    b.bin()
    assert b.run(d["merges"]) == d["merges"]
    check_against_digest(refpickle.build(b.checkpoint_state()), d, [k for k, _ in meta["merges"][: d["merges"]]])
    b.close()


def _canon(x, seen=None, skip=("_times", "save_dir", "parent", "rng")):
    """Structural form of a loaded checkpoint (refpickle records), cycles cut, timing fields dropped."""
    import math
    import numpy as np
    seen = {} if seen is None else seen  # id -> object: held, so no id is reused during the walk
    if isinstance(x, float):
        return "nan" if math.isnan(x) else round(x, 12)
    if isinstance(x, (str, int, bool)) or x is None:
        return x
    if hasattr(x, "to_numpy") and hasattr(x, "columns"):  # a pandas frame
        return [list(x.columns), _canon(x.to_numpy().tolist(), seen)]
    if isinstance(x, np.ndarray):
        return _canon(x.tolist(), seen)
    if id(x) in seen:
        return "<cycle>"
    seen[id(x)] = x
    if isinstance(x, dict):
        items = {str(k): _canon(v, seen) for k, v in x.items() if k not in skip}
        attrs = {k: _canon(v, seen) for k, v in getattr(x, "__dict__", {}).items() if k not in skip}
        return [type(x).__name__, sorted(items.items()), sorted(attrs.items())]
    if isinstance(x, (list, tuple)):
        return [_canon(v, seen) for v in x]
    if hasattr(x, "__dict__"):
        return [type(x).__name__, sorted((k, _canon(v, seen)) for k, v in vars(x).items() if k not in skip)]
    return repr(x)


def _first_diff(x, y, path="") -> str:
    if type(x) != type(y):
        return f"{path}: {type(x).__name__} != {type(y).__name__}"
    if isinstance(x, (list, tuple)):
        if len(x) != len(y):
            return f"{path}: len {len(x)} != {len(y)}"
        for i, (u, v) in enumerate(zip(x, y)):
            if u != v:
                return _first_diff(u, v, f"{path}/{u[0] if isinstance(u, tuple) and isinstance(u[0], str) else i}")
    return f"{path}: {str(x)[:300]} != {str(y)[:300]}"


@pytest.mark.gpu
def test_cli_two_ranks_write_the_single_gpu_checkpoint(tmp_path):
    """bin/encode.py under torchrun (2 ranks, gloo, sharing the one GPU): rows
    sharded, deltas exchanged per merge (pipelined), stats and the merge tree
    gathered to rank 0 -- the bpe_iter=*.pkl and stats equal the 1-GPU run's."""
    import os
    import socket
    import subprocess
    import sys
    from geobpe import refpickle
    cli = _encode_cli()
    common = ["--data-dir", "synthetic:300:30:150:5", "--bins", "1-5", "--save-every", "10", "--max-iter", "31"]
    one, two = tmp_path / "one", tmp_path / "two"
    assert cli.main(common + ["--save-dir", str(one), "--log-dir", str(tmp_path / "l1")]) == 0
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    here = os.path.dirname(os.path.abspath(__file__))
    enc = os.path.join(os.path.dirname(here), "pt-bpe_amd", "bin", "encode.py")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), enc] + common + \
        ["--save-dir", str(two), "--log-dir", str(tmp_path / "l2"), "--dist-backend", "gloo"]
    out = open(tmp_path / "ranks.out", "w")
    p = subprocess.Popen(cmd, stdout=out, stderr=subprocess.STDOUT, start_new_session=True)
    try:
        rc = p.wait(timeout=150)
    except subprocess.TimeoutExpired:
        os.killpg(p.pid, 9)  # torchrun and its workers (their own session)
        p.wait()
        rc = None
    out.close()
    log = (tmp_path / "ranks.out").read_text()[-3000:]
    elog = tmp_path / "l2" / "encode.log"
    assert rc == 0, log + (elog.read_text()[-2000:] if elog.exists() else "")
    for t in (10, 20, 30):
        a = refpickle.load(str(one / f"bpe_iter={t}.pkl"))
        b = refpickle.load(str(two / f"bpe_iter={t}.pkl"))
        assert refpickle.merge_keys(a) == refpickle.merge_keys(b) and len(refpickle.merge_keys(a)) == t + 1
        ca, cb = _canon(a), _canon(b)
        assert ca == cb, _first_diff(ca, cb)
        assert json.loads((one / f"stats={t}.json").read_text()) == json.loads((two / f"stats={t}.json").read_text())


def test_rank_gather_helpers():
    """Host logic of the multi-GPU checkpoint gather (no GPU): offsets concatenate,
    and per-rank merge events interleave merge by merge in rank (= slot) order."""
    import numpy as np
    from geobpe.bpe import BPE
    off = BPE._cat_offsets([np.array([0, 2, 5]), np.array([0, 1]), np.array([0, 3, 4, 6])])
    assert off.tolist() == [0, 2, 5, 6, 9, 10, 12]
    parts = [  # merge 0: rank 0 has slots 3, 7; rank 1 slot 2 (+ base 10); merge 1: rank 1 only
        {"a": np.array([3, 7]), "b": np.array([4, 8]), "eoff": np.array([0, 2, 2]), "base": 0},
        {"a": np.array([2, 5]), "b": np.array([3, 6]), "eoff": np.array([0, 1, 2]), "base": 10},
    ]
    a, b, eoff = BPE._merge_rank_events(parts)
    assert a.tolist() == [3, 7, 12, 15] and b.tolist() == [4, 8, 13, 16] and eoff.tolist() == [0, 3, 4]


def _utility_golden():
    import json
    import os
    from conftest import GOLDEN
    with open(os.path.join(GOLDEN, "codebook_utility.json")) as f:
        return json.load(f)


def _close(u, want):
    for k, v in want.items():
        assert abs(u[k] - v) <= 1e-5 * max(1.0, abs(v)), (k, u[k], v)


def test_codebook_utility_matches_reference_vectors():
    """get_codebook_utility against the reference function's own outputs
    (plotting.py:78-95 run in the build container: tests/golden/make_utility_golden.py)
    on the fixtures' encoded ids; float32 arithmetic, tolerance 1e-5 relative."""
    from conftest import load_golden
    from geobpe.bpe import get_codebook_utility
    for name, g in _utility_golden().items():
        ids = g["ids"] if "ids" in g else load_golden(name)[2]["ids"]
        _close(get_codebook_utility(ids, g["vocab_size"]), g["utility"])


@pytest.mark.gpu
def test_codebook_utility_of_device_encoding():
    """The stats of bin/encode.py (codebook utility of quantize(tokenize()) over every
    chain) on the HIP path's own encoding equal the reference's numbers."""
    from conftest import load_golden
    from geobpe.bpe import get_codebook_utility
    from geobpe.engine import GeoBPEEngine
    for name, g in _utility_golden().items():
        if "ids" in g:
            continue
        meta, corpus, _ = load_golden(name)
        eng = GeoBPEEngine(corpus, meta["bins"]["1"], device=0, strategy=meta.get("bin_strategy")).initialize()
        eng.bin()
        eng.run(len(meta["merges"]))
        ids, _ = eng.encode()
        assert eng.vocab_size == g["vocab_size"]
        _close(get_codebook_utility(ids, eng.vocab_size), g["utility"])
        eng.close()
