"""Golden fixtures for the RMSD-partitioned mode, made by running the
REFERENCE in this container (never on the GPU box; only the outputs travel).

The reference's `BPE` is run with a finite `rmsd_partition_min_size` (p), `res_init=True`,
`std_bonds=True`, `glue_opt=False` on small synthetic corpora.  Its RMSD paths need worker
pools (the `max_workers == 0` branches call `_compute_assignment` with four arguments,
`bpe.py:305,1767`, a TypeError), so this runs with SLURM_CPUS_PER_TASK=2.

Per fixture `<name>`:
  <name>.npz   the corpus, and the reference's per-chain geometry after initialize() and at
               the end (9 columns, float64) plus each chain's init triple
               (_init_n_ca, _init_ca_c, _init_bond_angle);
  <name>.json  the settings, the (flag, -count, key) popped at every step() entry (the
               reference's step() recurses for recurring keys, bpe.py:2164-2166), _step and
               len(_tokens) after each top-level call, _tokens, _sphere_dict keys, the
               segmentation [(start bond, id, #bonds)] per chain, quantize() of every chain
               (or the exception it raises), and what initialize/bin/step raised, if anything.

Usage: python tests/golden/make_rmsd_mode_golden.py [name ...]
"""
from __future__ import annotations

import json
import os
import subprocess
import sys
import tempfile
import traceback

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "pt-bpe_amd"))
sys.path.insert(0, HERE)

NUM_P = {2: 2, 3: 3, 5: 2, 8: 1}
# name: (n_chains, len_lo, len_hi, seed, B, p_min_size, super_res, max_num_strucs, step calls)
FIXTURES = {
    "rm_p0": (10, 20, 40, 21, 5, 0, False, 60, 25),
    "rm_p0_super": (10, 20, 40, 21, 5, 0, True, 60, 25),
    "rm_p3_super": (8, 15, 35, 22, 4, 3, True, 50, 20),
    "rm_p2_super_b3": (12, 10, 30, 23, 3, 2, True, 400, 30),
    "rm_p4": (6, 20, 30, 24, 5, 4, False, 60, 3),
    "rm_p0_b2_long": (16, 12, 30, 25, 2, 0, False, 80, 120),
    "rm_p0_super_b2_long": (16, 12, 30, 25, 2, 0, True, 80, 120),
    "rm_p0_b1_exhaust": (20, 10, 30, 26, 1, 0, False, 80, 250),
    # one partition per size and one bin: every residue alike, so equal geometry is built by
    # different merge orders and keys recur after their merge (bpe.py:1823-1847, 1862-1866)
    "rm_p0_b1_one_partition": (30, 6, 40, 27, 1, 0, False, 80, 400, {2: 1, 3: 1}),
    # multi-grid schedules (bins {size: B}): junctions of a key of L bonds are binned at
    # grid(L); the RMSD mode sets the medoid geometry before the neighbour keys, so the
    # keys stay consistent (unlike the scoped mode)
    "rm_p0_multigrid": (12, 20, 40, 28, {1: 5, 6: 3, 9: 4, 15: 2}, 0, False, 60, 60),
    "rm_p3_super_multigrid": (10, 15, 40, 29, {1: 4, 2: 6, 7: 6}, 3, True, 60, 40),
    # free bond lengths (--free-bonds, as in the README runs): bonds binned per grid too;
    # p = 3 raises KeyError in initialize() there
    "rm_p0_super_freebonds": (10, 20, 40, 30, 5, 0, True, 60, 40, NUM_P, False),
    "rm_p2_freebonds_multigrid": (12, 15, 35, 31, {1: 4, 6: 3}, 2, False, 60, 40, NUM_P, False),
    "rm_p3_freebonds": (6, 15, 30, 32, 5, 3, False, 60, 5, NUM_P, False),
    # no RMSD partitioning (p = inf) with a multi-grid schedule: the reference's step()
    # re-snaps after computing the neighbour keys, its stored keys go stale and, with
    # breakpoints off, it skips those occurrences (bpe.py:1909-1920) -- its own semantics,
    # recorded here
    "rm_pinf_multigrid": (20, 30, 80, 33, {1: 5, 2: 6, 3: 8, 5: 4, 6: 7, 9: 5, 12: 3, 15: 1}, float("inf"),
                          False, 60, 30),
    # config 1's corpus (every PDB of the reference's data/vqvae_pretrain/train, featurised by
    # pdb_angles.py) in the README's first run minus glue optimisation: --bins 1-50, p = 0,
    # --num-p 2-2:3-5:5-1:6-2:8-1, max_num_strucs 500, free bonds, rmsd_super_res
    "rm_pdb72_readme": ("pdb72", None, None, 0, 50, 0, True, 500, 20, {2: 2, 3: 5, 5: 1, 6: 2, 8: 1}, False),
    # one chain: its last residue is the only size-2 structure, k_medoids returns [0] and the
    # reference's memmap write of num_partitions[2] = 2 entries broadcasts that one medoid
    # (bpe.py:298-300); the run carries on with one size-2 partition
    "rm_p0_one_chain": (1, 30, 40, 34, 5, 0, False, 60, 20),
    # rmsd_only (bpe.py:1977, 2027): a partitioned merge keeps its own geometry (no medoid
    # written over it), so later keys see the chains' raw values
    "rm_p0_rmsd_only": (10, 20, 40, 21, 5, 0, False, 60, 25),
    "rm_p3_super_rmsd_only": (8, 15, 35, 22, 4, 3, True, 50, 20),
    "rm_p0_b2_long_rmsd_only": (16, 12, 30, 25, 2, 0, False, 80, 120),
    # bond-level init (res_init=False): every bond its own token, pairs of bonds first
    "rm_p0_bondinit": (8, 15, 30, 35, 5, 0, False, 60, 40),
    "rm_p3_super_bondinit": (8, 15, 30, 36, 4, 3, True, 60, 40),
    "rm_pinf_bondinit": (8, 15, 30, 37, 5, float("inf"), False, 60, 40),
    "rm_pinf_bondinit_b3_long": (12, 20, 40, 38, 3, float("inf"), False, 60, 250),
}
# further BPE(...) arguments of a fixture
EXTRA = {n: {"rmsd_only": True} for n in FIXTURES if n.endswith("_rmsd_only")}
# bond-level init (res_init=False, bpe.py:397-420): every bond its own initial token
EXTRA.update({n: {"res_init": False} for n in FIXTURES if "_bondinit" in n})
# BPE.tokenize (bpe.py:1053-1140, the RMSD mode's induce) after the training calls, on: the
# first three training chains, the first 60 % of chains 3 and 4 (values inside the trained
# bins), and new synthetic chains (chains, len_lo, len_hi, seed) -- those usually hold a value
# outside the trained range, and the reference's get_ind raises ValueError (recorded).  It
# needs the residue partitions of both sizes (p <= 2: it skips the first two _sphere_dict
# keys, :1116-1119)
INDUCE = {
    "rm_p0": (5, 15, 45, 99),
    "rm_p0_super": (5, 15, 45, 98),
    "rm_p2_super_b3": (6, 10, 30, 97),
    "rm_p0_super_freebonds": (5, 15, 45, 96),
    "rm_pdb72_readme": (4, 40, 120, 95),
    # rmsd_only: step_helper keeps each occurrence's own geometry (bpe.py:1386)
    "rm_p0_rmsd_only": (5, 15, 45, 94),
    "rm_p0_b2_long_rmsd_only": (5, 12, 30, 93),
}
COLS = ["0C:1N", "N:CA", "CA:C", "phi", "psi", "omega", "tau", "CA:C:1N", "C:1N:1CA"]


def _id(v):
    return [int(x) for x in v] if isinstance(v, tuple) else int(v)


def run_one(name):
    import numpy as np
    from geobpe import synth
    from make_golden import _stub_optional_deps

    nch, lo, hi, seed, B, p, sup, maxs, calls = FIXTURES[name][:9]
    num_p = FIXTURES[name][9] if len(FIXTURES[name]) > 9 else NUM_P
    std = FIXTURES[name][10] if len(FIXTURES[name]) > 10 else True
    if nch == "pdb72":
        import pdb_angles
        corpus, _ = pdb_angles.pdb_dir_corpus("/root/reference/data/vqvae_pretrain/train")
        nch = len(corpus["row_off"]) - 1
    else:
        corpus = synth.make_corpus(synth.make_lengths(nch, lo, hi, seed=seed), seed=seed)
    _stub_optional_deps()
    sys.path.insert(0, "/root/reference")
    import foldingdiff.bpe as RB
    from foldingdiff.tokenizer import Tokenizer

    RB.BPE.visualize = lambda self, key, path: None
    Tokenizer.visualize_bonds = lambda self, *a, **k: None
    popped = []
    inner_step = RB.BPE.step

    def recording_step(self):
        top = self._priority_dict.peekitem(0)[0]
        popped.append([bool(top[0]), int(top[1]), top[2]])
        return inner_step(self)

    RB.BPE.step = recording_step
    structs = []
    for i, row in enumerate(synth.corpus_rows(corpus)):
        s = Tokenizer.init_structure(len(row["phi"]))
        for c in COLS:
            s["angles"][c] = row[c].astype(np.float64)
        s["fname"] = f"synthetic_{i}"
        structs.append(s)

    def geometry(bpe, tag, arrays):
        for c in COLS:
            arrays[f"{tag}_{c}"] = np.concatenate(
                [np.array([float(x) for x in t.angles_and_dists[c]]) for t in bpe.tokenizers])
        arrays[f"{tag}_init"] = np.array([[float(t._init_n_ca), float(t._init_ca_c), float(t._init_bond_angle)]
                                          for t in bpe.tokenizers])

    def segmentation(bpe):
        return [[[int(s), _id(v[1]), int(v[2])] for s, v in t.bond_to_token.items()] for t in bpe.tokenizers]

    bins = dict(B) if isinstance(B, dict) else {1: B}
    meta = {"name": name, "n_chains": nch, "len_lo": lo, "len_hi": hi, "seed": seed,
            "bins": {str(k): v for k, v in bins.items()},
            "rmsd_partition_min_size": p, "rmsd_super_res": sup, "max_num_strucs": maxs, "std_bonds": std,
            "num_partitions": {str(k): v for k, v in num_p.items()}, "rng_seed": 0, "calls": [],
            "extra": EXTRA.get(name, {}),
            "raised": None, "generator": "tests/golden/make_rmsd_mode_golden.py (reference: /root/reference "
                                         "foldingdiff/bpe.py, run in the build container)"}
    arrays = dict(corpus)
    bpe = RB.BPE(structs, bins=bins, save_dir=tempfile.mkdtemp(prefix="geobpe_rmsd_golden_"),
                 rmsd_partition_min_size=p, rmsd_super_res=sup, num_partitions=dict(num_p),
                 max_num_strucs=maxs, std_bonds=std, seed=0, **({"res_init": True} | EXTRA.get(name, {})))
    try:
        bpe.initialize()
        geometry(bpe, "init", arrays)
        meta["init_tokens"] = [[_id(k), v] for k, v in bpe._tokens.items()]
        meta["init_segmentation"] = segmentation(bpe)
        meta["init_sphere_keys"] = list(getattr(bpe, "_sphere_dict", {}) or {})
        bpe.bin()
        meta["bin_keys"] = len(bpe._priority_dict)
        meta["bin_top"] = [[bool(a), int(b), c] for (a, b, c) in list(bpe._priority_dict.keys())[:20]]
        for _ in range(calls):
            if len(bpe._priority_dict) == 0:
                break
            n0 = len(popped)
            bpe.step()
            meta["calls"].append({"popped": popped[n0:], "step": bpe._step, "n_tokens": len(bpe._tokens)})
    except BaseException as e:  # noqa: BLE001 - the fixture records what the reference raises
        meta["raised"] = {"type": type(e).__name__, "msg": str(e)[:300], "popped_so_far": popped[-1:],
                          "where": traceback.format_exc().splitlines()[-4:]}
    if name in INDUCE and not meta["raised"]:
        run_induce(name, bpe, Tokenizer, RB, meta, arrays, corpus)
    if "init_tokens" in meta:
        geometry(bpe, "final", arrays)
        meta["tokens"] = [[_id(k), v] for k, v in bpe._tokens.items()]
        meta["sphere_keys"] = list(getattr(bpe, "_sphere_dict", {}) or {})
        meta["segmentation"] = segmentation(bpe)
        meta["step"] = bpe._step
        q = []
        for t in bpe.tokenizers:
            try:
                q.append([int(x) for x in bpe.quantize(t)])
            except Exception as e:  # noqa: BLE001
                q.append({"raised": type(e).__name__})
        meta["quantize"] = q
        meta["vocab_size"] = bpe.vocab_size
        if getattr(bpe, "_priority_dict", None):
            meta["final_top"] = [[bool(a), int(b), c] for (a, b, c) in list(bpe._priority_dict.keys())[:20]]
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **arrays)
    with open(os.path.join(HERE, f"{name}.json"), "w") as f:
        json.dump(meta, f)
    merges = sum(len(c["popped"]) for c in meta["calls"])
    print(f"{name}: calls={len(meta['calls'])} merges={merges} step={meta.get('step')} "
          f"raised={meta['raised'] and meta['raised']['type']}", flush=True)


class _Chain:  # esm's ProteinChain stand-in: the metrics it feeds (bb RMSD, lDDT) are not recorded
    @classmethod
    def from_pdb(cls, *a, **k):
        return cls()

    @classmethod
    def from_backbone_atom_coordinates(cls, *a, **k):
        return cls()

    def rmsd(self, *a, **k):
        return 0.0

    def lddt_ca(self, *a, **k):
        import numpy as np
        return np.zeros(1)


def induce_corpus(train, name):
    """The chains run_induce tokenizes (see INDUCE), as one corpus."""
    import numpy as np
    from geobpe import synth
    n_new, lo, hi, seed = INDUCE[name]
    ro = train["row_off"]
    rows = []
    for r in range(5):
        a, b = int(ro[r]), int(ro[r + 1])
        if r >= 3:
            b = a + max(2, int(0.6 * (b - a)))
        rows.append({c: np.array(train[c][a:b], dtype=np.float64) for c in COLS})
        if r >= 3:  # the reference's padding at the new end (angles_and_coords.py:101-149)
            for c in ["psi", "omega", "tau", "CA:C:1N", "C:1N:1CA"]:
                rows[-1][c][-1] = np.nan
            for c in ["0C:1N", "N:CA", "CA:C"]:
                rows[-1][c][-1] = 0.0
    new = synth.make_corpus(synth.make_lengths(n_new, lo, hi, seed=seed), seed=seed)
    rows += list(synth.corpus_rows(new))
    out = {c: np.concatenate([x[c] for x in rows]) for c in COLS}
    out["row_off"] = np.concatenate([[0], np.cumsum([len(x["phi"]) for x in rows])]).astype(np.int64)
    return out, rows


def run_induce(name, bpe, Tokenizer, RB, meta, arrays, train):
    import numpy as np
    corpus, rows = induce_corpus(train, name)
    for c in COLS + ["row_off"]:
        arrays[f"new_{c}"] = corpus[c]
    RB.ProteinChain = _Chain
    out = []
    for i, row in enumerate(rows):
        s = Tokenizer.init_structure(len(row["phi"]))
        for c in COLS:
            s["angles"][c] = row[c]
        s["fname"] = f"new_{i}"
        try:
            t, metrics = bpe.tokenize(Tokenizer(s))
        except Exception as e:  # noqa: BLE001 - recorded: the reference's behaviour on this chain
            out.append({"raised": type(e).__name__, "msg": str(e)[:200]})
            continue
        out.append({"segmentation": [[int(a), _id(v[1]), int(v[2])] for a, v in t.bond_to_token.items()],
                    "L": [int(x) for x in metrics["L"]]})
        for c in COLS:
            arrays[f"new{i}_{c}"] = np.array([float(x) for x in t.angles_and_dists[c]])
        arrays[f"new{i}_init"] = np.array([float(t._init_n_ca), float(t._init_ca_c), float(t._init_bond_angle)])
    meta["induce"] = out


def main(argv):
    if len(argv) >= 2 and argv[0] == "--one":
        run_one(argv[1])
        return
    env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1", MPLBACKEND="Agg", SLURM_CPUS_PER_TASK="2",
               PYTHONBREAKPOINT="0")
    for name in argv or list(FIXTURES):
        r = subprocess.run([sys.executable, "-W", "ignore", __file__, "--one", name], env=env,
                           stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
        out = [ln for ln in r.stdout.splitlines() if ln.startswith(name + ":")]
        print(out[-1] if out and r.returncode == 0 else f"{name}: rc={r.returncode} {r.stderr[-800:]}", flush=True)


if __name__ == "__main__":
    main(sys.argv[1:])
