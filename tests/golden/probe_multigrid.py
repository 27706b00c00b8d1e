"""Record what the REFERENCE does with a multi-grid ``--bins`` schedule (SURVEY.md
§8(f) row 3) in the scoped mode, as evidence for DESIGN.md §7.

Run only in the build container (it imports /root/reference); writes
``tests/golden/multigrid_reference.json``.

Finding: ``BPE.step`` computes the new neighbour keys (step 5,
foldingdiff/bpe.py:1990-2006) BEFORE it re-snaps the merged span to the bin
centres of grid(|token|) (step 6, bpe.py:2010-2013).  With one grid the re-snap is
idempotent; with several it changes the values, so the stored neighbour keys differ
from what ``compute_geo_key`` later recomputes (bpe.py:1917-1920, "should never
happen" -> ``breakpoint()``).  Interactively that opens the debugger; with stdin at
EOF pdb raises BdbQuit; with PYTHONBREAKPOINT=0 the occurrence is skipped, stays in
``_geo_dict[key]``, and every later step re-selects the same key without merging
anything (a new token id per step).

The same file records the free-bonds case (std_bonds=False): the reference raises
KeyError('N:CA') in initialize() (see run_free_bonds).

Usage:  python tests/golden/probe_multigrid.py
"""
from __future__ import annotations

import builtins
import inspect
import json
import os
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
BINS = {1: 5, 2: 6, 3: 8, 5: 4, 6: 7, 9: 5, 12: 3, 15: 1}
SHAPE = dict(n_seqs=60, len_lo=30, len_hi=110, seed=9, repeat_frac=0.2)
MERGES = 8


def run(mode: str) -> dict:
    if mode == "free-bonds":
        return run_free_bonds()
    sys.path.insert(0, HERE)
    import numpy as np
    import make_golden
    from geobpe import synth

    make_golden._stub_optional_deps()
    sys.path.insert(0, "/root/reference")
    import foldingdiff.bpe as B
    from foldingdiff.tokenizer import Tokenizer

    B.BPE.visualize = lambda self, key, path: None
    hits = []

    def on_breakpoint():  # the reference's breakpoint() calls, recorded
        f = inspect.currentframe().f_back
        L = f.f_locals
        rec = {"line": f.f_lineno, "step": L["self"]._step}
        if "geo_key" in L and "key" in L:
            k, g = json.loads(L["key"]), json.loads(L["geo_key"])
            rec["differs"] = {t: [k[t], g[t]] for t in k if k[t] != g[t]}
        hits.append(rec)
        if mode == "debugger":
            raise RuntimeError("breakpoint")

    builtins.breakpoint = on_breakpoint
    lengths = synth.make_lengths(SHAPE["n_seqs"], SHAPE["len_lo"], SHAPE["len_hi"], seed=SHAPE["seed"])
    corpus = synth.make_corpus(lengths, seed=SHAPE["seed"], repeat_frac=SHAPE["repeat_frac"])
    structs = []
    for i, row in enumerate(synth.corpus_rows(corpus)):
        s = Tokenizer.init_structure(len(row["phi"]))
        for c in synth.COLUMNS:
            s["angles"][c] = row[c].astype(np.float64)
        s["fname"] = f"synthetic_{i}"
        structs.append(s)
    bpe = B.BPE(structs, bins=dict(BINS), bin_strategy="histogram", save_dir=tempfile.mkdtemp(prefix="geobpe_mg_"),
                rmsd_partition_min_size=float("inf"), res_init=True, std_bonds=True, seed=0)
    bpe.initialize()
    bpe.bin()
    merges = []
    err = None
    for _ in range(MERGES):
        (_, negc, key), _ = bpe._priority_dict.peekitem(0)
        tokens = sum(len(t.bond_to_token) for t in bpe.tokenizers)
        merges.append({"key": key, "count": -negc, "live_tokens_before": tokens})
        try:
            bpe.step()
        except RuntimeError as e:
            err = f"{e} at step {bpe._step}"
            break
    return {"mode": mode, "merges": merges, "breakpoints": hits[:4], "n_breakpoints": len(hits), "stopped": err,
            "vocab_size_after": len(bpe._tokens)}


def run_free_bonds() -> dict:
    """std_bonds=False with res_init=True: quant_geo bins the bond lengths through the
    top-level ``_thresholds[bond]`` entries (bpe.py:1518-1519), which only std_bonds
    creates (bpe.py:874-876) -> KeyError('N:CA') inside initialize()."""
    sys.path.insert(0, HERE)
    import numpy as np
    import make_golden
    from geobpe import synth

    make_golden._stub_optional_deps()
    sys.path.insert(0, "/root/reference")
    import foldingdiff.bpe as B
    from foldingdiff.tokenizer import Tokenizer

    lengths = synth.make_lengths(10, 30, 60, seed=11)
    corpus = synth.make_corpus(lengths, seed=11)
    structs = []
    for i, row in enumerate(synth.corpus_rows(corpus)):
        s = Tokenizer.init_structure(len(row["phi"]))
        for c in synth.COLUMNS:
            s["angles"][c] = row[c].astype(np.float64)
        s["fname"] = f"synthetic_{i}"
        structs.append(s)
    bpe = B.BPE(structs, bins={1: 3}, bin_strategy="histogram", save_dir=tempfile.mkdtemp(prefix="geobpe_fb_"),
                rmsd_partition_min_size=float("inf"), res_init=True, std_bonds=False, seed=0)
    try:
        bpe.initialize()
        return {"mode": "free-bonds", "raised": None}
    except Exception as e:  # the reference's own error, recorded
        return {"mode": "free-bonds", "raised": type(e).__name__, "args": [str(a) for a in e.args]}


def main():
    if len(sys.argv) == 3 and sys.argv[1] == "--one":
        print("RESULT " + json.dumps(run(sys.argv[2])))
        return
    env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1", MPLBACKEND="Agg", SLURM_CPUS_PER_TASK="0")
    out = {"bins": {str(k): v for k, v in BINS.items()}, "corpus": SHAPE,
           "generator": "tests/golden/probe_multigrid.py (reference: /root/reference foldingdiff/bpe.py)"}
    for mode in ("debugger", "PYTHONBREAKPOINT=0", "free-bonds"):
        r = subprocess.run([sys.executable, "-W", "ignore", __file__, "--one", mode], env=env, check=True,
                           stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, text=True, stdin=subprocess.DEVNULL)
        line = [x for x in r.stdout.splitlines() if x.startswith("RESULT ")][-1]
        out[mode] = json.loads(line[len("RESULT "):])
    with open(os.path.join(HERE, "multigrid_reference.json"), "w") as f:
        json.dump(out, f, indent=1)
    for mode in ("debugger", "PYTHONBREAKPOINT=0"):
        r = out[mode]
        print(mode, "merges", [(m["count"], m["live_tokens_before"]) for m in r["merges"]], "breakpoints",
              r["n_breakpoints"], "stopped", r["stopped"])


if __name__ == "__main__":
    main()
