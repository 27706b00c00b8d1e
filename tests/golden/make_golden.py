"""Generate golden parity fixtures by running the REFERENCE GeoBPE in this container.

Run only in the build container (``/root/reference`` does not exist on the GPU
box); the outputs under ``tests/golden/`` are small data files that travel.

Recipe: SURVEY.md Appendix B.  The reference's optional plotting/PDB deps
(biotite, esm, seaborn, astropy, imageio) are stubbed in ``sys.modules``; they are
not touched in the scoped mode (res_init=True, p_min_size=inf, glue_opt=False,
bin_strategy=histogram, std_bonds=True).  ``BPE.visualize`` only renders PNGs
(`foldingdiff/bpe.py:1583-1627`) and is patched to a no-op.

Per fixture ``<name>`` this writes
  <name>.npz   inputs (the synthetic corpus, `geobpe.synth` layout) and the
               numeric outputs: init labels, final segmentation, encoded ids;
  <name>.json  bins, thresholds, merge list [(key, count)], vocab (`_tokens`),
               vocab_size, K0.

Usage:  python tests/golden/make_golden.py [name ...]
"""
from __future__ import annotations

import json
import os
import subprocess
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "pt-bpe_amd"))
sys.path.insert(0, HERE)

# name: (n_seqs, len_lo, len_hi, bins, merges, seed, repeat_frac)
FIXTURES = {
    "g40x50_b5": (40, 50, None, 5, 60, 0, 0.0),
    "g30x40-120_b2": (30, 40, 120, 2, 200, 1, 0.0),
    "g40x40-120_b12": (40, 40, 120, 12, 120, 2, 0.0),
    "g60x20-90_b5_rep": (60, 20, 90, 5, 150, 3, 0.25),
    "g25x1-12_b3_short": (25, 1, 12, 3, 40, 4, 0.0),
    "g300x60-200_b5": (300, 60, 200, 5, 40, 5, 0.0),
    "g80x40-160_b7_rep": (80, 40, 160, 7, 100, 6, 0.1),
    "g50x30-110_b6_cover": (50, 30, 110, 6, 80, 7, 0.1, "histogram-cover"),
    "g50x30-110_b5_uniform": (50, 30, 110, 5, 80, 8, 0.1, "uniform"),
    # config 1 shape: the bundled PDB subset (tests/golden/pdb, from the reference's
    # data/vqvae_pretrain/train) featurised by pdb_angles.py, 5 bins, 50 merges
    "c1_pdb12_b5": ("pdb", None, None, 5, 50, 0, 0.0),
    # config 1 at its stated size: every PDB of the reference's data/vqvae_pretrain/train
    # (72 files, read here at generation time; only the featurised angles travel)
    "c1_pdb72_b5": ("pdb72", None, None, 5, 50, 0, 0.0),
}
PDB72 = "/root/reference/data/vqvae_pretrain/train"


def _stub_optional_deps():
    import types

    class _D:
        def __init__(s, *a, **k):
            pass

        def __call__(s, *a, **k):
            return _D()

        def __getattr__(s, n):
            return _D()

    class _M(types.ModuleType):
        def __getattr__(s, n):
            if n.startswith("__"):
                raise AttributeError(n)
            return _D

    for n in ["biotite", "biotite.structure", "biotite.structure.io", "biotite.structure.io.pdb",
              "biotite.sequence", "biotite.sequence.align", "seaborn", "esm", "esm.utils",
              "esm.utils.structure", "esm.utils.structure.protein_chain", "astropy",
              "astropy.visualization", "astropy.visualization.mpl_normalize", "imageio"]:
        m = _M(n)
        m.__path__ = []
        sys.modules[n] = m


def run_one(name: str) -> None:
    import numpy as np
    from geobpe import synth

    n_seqs, lo, hi, bins, merges, seed, rep = FIXTURES[name][:7]
    strategy = FIXTURES[name][7] if len(FIXTURES[name]) > 7 else "histogram"
    if n_seqs in ("pdb", "pdb72"):
        import pdb_angles
        corpus, _ = pdb_angles.pdb_dir_corpus(os.path.join(HERE, "pdb") if n_seqs == "pdb" else PDB72)
        n_seqs = len(corpus["row_off"]) - 1
    else:
        lengths = synth.make_lengths(n_seqs, lo, hi, seed=seed)
        corpus = synth.make_corpus(lengths, seed=seed, repeat_frac=rep)

    _stub_optional_deps()
    sys.path.insert(0, "/root/reference")
    import foldingdiff.bpe as B
    from foldingdiff.tokenizer import Tokenizer

    B.BPE.visualize = lambda self, key, path: None
    structs = []
    for i, row in enumerate(synth.corpus_rows(corpus)):
        n = len(row["phi"])
        s = Tokenizer.init_structure(n)
        for c in synth.COLUMNS:
            s["angles"][c] = row[c].astype(np.float64)
        s["fname"] = f"synthetic_{i}"
        structs.append(s)
    t0 = time.time()
    bpe = B.BPE(structs, bins={1: bins}, bin_strategy=strategy, save_dir=tempfile.mkdtemp(prefix="geobpe_golden_"),
                rmsd_partition_min_size=float("inf"), res_init=True, std_bonds=True, seed=0)
    bpe.initialize()
    init_labels = np.concatenate([
        np.array([v[1] for v in t.bond_to_token.values()], dtype=np.int64) for t in bpe.tokenizers])
    k0 = len(bpe._tokens)
    t1 = time.time()
    bpe.bin()
    t2 = time.time()
    merge_list = []
    for _ in range(merges):
        if len(bpe._priority_dict) == 0:
            break
        (_, negc, key), _ = bpe._priority_dict.peekitem(0)
        merge_list.append([key, -negc])
        bpe.step()
    t3 = time.time()
    seg_start, seg_id, seg_off = [], [], [0]
    ids, ids_off = [], [0]
    for t in bpe.tokenizers:
        for s, v in t.bond_to_token.items():
            seg_start.append(s // 3)
            seg_id.append(v[1])
        seg_off.append(len(seg_start))
        q = bpe.quantize(t)
        ids.extend(q)
        ids_off.append(len(ids))
    thresholds = {k: [list(p) for p in v] for k, v in bpe._thresholds[1].items()}
    # object-API views for the host mirror (geobpe.bpe): first three chains
    t0s = bpe.tokenizers[:3]
    api = {
        "tokenize": [[list(x) for x in t.tokenize()] for t in t0s],
        "token_pos": [list(t.token_pos) for t in t0s],
        "bond_to_token": [[list(v) for v in t.bond_to_token.values()] for t in t0s],
        "dequantize": [[list(x) for x in bpe.dequantize(bpe.quantize(t))] for t in t0s],
        "recover": [bpe.recover(t.tokenize()) for t in t0s],
        "capacity": bpe.capacity(), "capacity_tokenizer": float(bpe.capacity(tokenizer=True)),
        "bin_counts": {k: [int(c) for c in v] for k, v in bpe._bin_counts[1].items()},
    }
    meta = {
        "name": name,
        "n_seqs": n_seqs, "len_lo": lo, "len_hi": hi, "seed": seed, "repeat_frac": rep,
        "bins": {"1": bins},
        "bin_strategy": strategy,
        "api": api,
        "merges_requested": merges,
        "K0": k0,
        "thresholds": thresholds,
        "merges": merge_list,
        "vocab": {str(k): v for k, v in bpe._tokens.items()},
        "vocab_size": bpe.vocab_size,
        "cum_bin_count": {k: bpe.cum_bin_count(k) for k in ["C:1N:1CA", "omega", "phi"]},
        "reference_seconds": {"initialize": t1 - t0, "bin": t2 - t1, "steps": t3 - t2},
        "generator": "tests/golden/make_golden.py (reference: /root/reference foldingdiff/bpe.py)",
    }
    np.savez_compressed(
        os.path.join(HERE, f"{name}.npz"),
        **corpus,
        init_labels=init_labels,
        seg_start=np.array(seg_start, dtype=np.int64), seg_id=np.array(seg_id, dtype=np.int64),
        seg_off=np.array(seg_off, dtype=np.int64),
        ids=np.array(ids, dtype=np.int64), ids_off=np.array(ids_off, dtype=np.int64),
    )
    with open(os.path.join(HERE, f"{name}.json"), "w") as f:
        json.dump(meta, f)
    print(f"{name}: K0={k0} merges={len(merge_list)} init={t1-t0:.1f}s bin={t2-t1:.1f}s "
          f"steps={t3-t2:.1f}s", flush=True)


def main(argv):
    if len(argv) >= 2 and argv[0] == "--one":
        run_one(argv[1])
        return
    names = argv or list(FIXTURES)
    env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1", MPLBACKEND="Agg", SLURM_CPUS_PER_TASK="0")
    for name in names:
        r = subprocess.run([sys.executable, "-W", "ignore", __file__, "--one", name], env=env, check=True,
                           stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, text=True)
        print(r.stdout.strip().splitlines()[-1], flush=True)


if __name__ == "__main__":
    main(sys.argv[1:])
