"""Merge replay (bin/induce.py; geobpe.induce): a trained vocabulary applied to
chains in training order.  CPU: the vocabulary decoding against the reference's
own fixtures and the replay definition on the oracle.  GPU: the HIP replay
(k_select_replay) against the oracle's replay, and the training segmentation
reproduced on the training corpus."""
import numpy as np
import pytest

from conftest import golden_names, load_golden

ANGLES = ["tau", "CA:C:1N", "C:1N:1CA", "psi", "omega", "phi"]


@pytest.mark.parametrize("name", golden_names())
def test_vocabulary_decodes_reference_tokens(name, oracle_lib):
    """_tokens of the reference -> residue symbols (== the oracle's labels) and
    merged contents whose key strings are the reference's merge list."""
    from geobpe import induce
    meta, corpus, _ = load_golden(name)
    B = meta["bins"]["1"]
    thr = {k: [tuple(p) for p in v] for k, v in meta["thresholds"].items()}
    sol, K0, contents = induce.vocabulary(induce.tokens_from_json(meta["vocab"]), thr, B)
    o = oracle_lib.OracleBPE(corpus, B, cover=meta.get("bin_strategy") == "histogram-cover",
                             strategy=meta.get("bin_strategy")).initialize()
    assert K0 == meta["K0"] and np.array_equal(sol, o.sym_of_label)
    assert induce.merge_keys_of(contents, K0, B) == [k for k, _ in meta["merges"]]
    rec = induce.replay_records(contents, K0)
    for t in range(len(contents) - K0):  # the split concatenates to the content
        a, g, b = int(rec["idL"][t]), int(rec["g"][t]), int(rec["idR"][t])
        assert contents[a] + (g,) + contents[b] == contents[K0 + t] and a < K0 + t and b < K0 + t


def held_out(corpus_train, thr, sol, B, n, seed):
    """Chains from the same generator, angles clipped into the trained ranges,
    keeping chains whose residue geometries are all in the vocabulary."""
    from geobpe import synth
    from geobpe.dist import slice_corpus
    from oracle import prologue
    c = synth.make_corpus(synth.make_lengths(n, 20, 160, seed=seed), seed=seed)
    for k in ANGLES:
        v = c[k].copy()
        ok = ~np.isnan(v) & (v != 0)
        w = (v[ok] + 2 * np.pi) % (2 * np.pi)
        v[ok] = np.clip(w, thr[k][0][0], thr[k][-1][1])
        c[k] = v
    rsym, _ = prologue.symbols(c, thr, B)
    known = np.isin(rsym, sol)
    ro = c["row_off"]
    keep = [r for r in range(n) if known[ro[r]:ro[r + 1]].all()]
    parts = [slice_corpus(c, r, r + 1) for r in keep]
    out = {k: np.concatenate([p[k] for p in parts]) for k in synth.COLUMNS}
    out["row_off"] = np.concatenate([[0], np.cumsum([p["row_off"][-1] for p in parts])]).astype(np.int64)
    return out


def oracle_replay(oracle_lib, corpus, thr, sol, B, rec):
    o = oracle_lib.OracleBPE(corpus, B, thresholds=thr, sym_of_label=sol).initialize()
    o.bin()
    for t in range(len(rec["idL"])):
        n, _ = o.step_forced(rec["idL"][t], rec["g"][t], rec["idR"][t])
        assert n == o.K0 + t
    return o


def _train(oracle_lib, corpus, B, M):
    o = oracle_lib.OracleBPE(corpus, B).initialize()
    o.bin()
    for _ in range(M):
        assert o.step() is not None
    return o


def test_oracle_replay_reproduces_training(oracle_lib):
    from geobpe import induce, synth
    corpus = synth.make_corpus(synth.make_lengths(300, 20, 150, seed=81), seed=81, repeat_frac=0.1)
    o = _train(oracle_lib, corpus, 5, 150)
    sol, K0, contents = induce.vocabulary(o.vocab(), o.thresholds, 5)
    r = oracle_replay(oracle_lib, corpus, o.thresholds, sol, 5, induce.replay_records(contents, K0))
    for x, y in zip(r.segmentation(), o.segmentation()):
        assert np.array_equal(x, y)
    assert [c for _, c in r.merges] == [c for _, c in o.merges]


def test_replay_rejects_unknown_residue_geometry(oracle_lib):
    from geobpe import synth
    corpus = synth.make_corpus(synth.make_lengths(50, 20, 60, seed=82), seed=82)
    o = _train(oracle_lib, corpus, 5, 5)
    with pytest.raises(ValueError):
        oracle_lib.OracleBPE(corpus, 5, thresholds=o.thresholds, sym_of_label=o.sym_of_label[:3]).initialize()


@pytest.mark.gpu
def test_gpu_replay_reproduces_training_segmentation(oracle_lib):
    from geobpe import induce, synth
    corpus = synth.make_corpus(synth.make_lengths(3000, 20, 300, seed=83), seed=83, repeat_frac=0.05)
    o = _train(oracle_lib, corpus, 5, 300)
    eng = induce.induce(corpus, o.vocab(), o.thresholds, 5)
    for x, y in zip(eng.segmentation(), o.segmentation()):
        assert np.array_equal(x, y)
    for x, y in zip(eng.encode(), o.encode()):
        assert np.array_equal(x, y)
    assert [m[1] for m in eng.merges] == [c for _, c in o.merges]  # replayed counts
    a, b, off = eng.events()
    oa, ob, ooff = o.events()
    assert np.array_equal(off, ooff)
    eng.close()


@pytest.mark.gpu
@pytest.mark.parametrize("B, M", [(5, 400), (3, 200), (7, 150)])
def test_gpu_replay_on_new_chains_matches_oracle(oracle_lib, B, M):
    from geobpe import induce, synth
    train = synth.make_corpus(synth.make_lengths(1500, 20, 200, seed=84 + B), seed=84 + B, repeat_frac=0.05)
    o = _train(oracle_lib, train, B, M)
    sol, K0, contents = induce.vocabulary(o.vocab(), o.thresholds, B)
    rec = induce.replay_records(contents, K0)
    new = held_out(train, o.thresholds, sol, B, 800, seed=184 + B)
    r = oracle_replay(oracle_lib, new, o.thresholds, sol, B, rec)
    eng = induce.induce(new, o.vocab(), o.thresholds, B)
    assert eng.K0 == K0
    for x, y in zip(eng.segmentation(), r.segmentation()):
        assert np.array_equal(x, y)
    for x, y in zip(eng.encode(), r.encode()):
        assert np.array_equal(x, y)
    assert [m[1] for m in eng.merges] == [c for _, c in r.merges]
    eng.close()


@pytest.mark.gpu
def test_induce_cli_roundtrip(tmp_path):
    """bin/encode.py trains and checkpoints; bin/induce.py tokenizes the same
    corpus from the checkpoint: the tokenizers equal the checkpoint's own."""
    import importlib.util
    import json
    import os
    from conftest import REPO
    from geobpe import refpickle

    def cli(name):
        spec = importlib.util.spec_from_file_location(f"geobpe_{name}_cli", os.path.join(REPO, "pt-bpe_amd", "bin",
                                                                                       f"{name}.py"))
        m = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(m)
        return m
    data = "synthetic:200:20:120:7"
    enc = cli("encode")
    assert enc.main(["--data-dir", data, "--bins", "1-5", "--save-every", "20", "--max-iter", "41",
                     "--save-dir", str(tmp_path / "train"), "--log-dir", str(tmp_path / "logs")]) == 0
    src = str(tmp_path / "train" / "bpe_iter=40.pkl")
    ind = cli("induce")
    assert ind.main(["--src-pkl", src, "--data-dir", data, "--save-dir", str(tmp_path / "ind")]) == 0
    a, b = refpickle.load(src), refpickle.load(str(tmp_path / "ind" / "bpe_iter=40.pkl"))
    assert len(a.tokenizers) == len(b.tokenizers) == 200
    for x, y in zip(a.tokenizers, b.tokenizers):
        assert dict(x._bond_to_token) == dict(y._bond_to_token)
    u = json.loads((tmp_path / "ind" / "utility.json").read_text())
    assert 0 < u["use_ratio"] <= 1
