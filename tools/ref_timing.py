"""Time the REFERENCE GeoBPE (foldingdiff/bpe.py) in this container on subsets of
the C3 corpus (SURVEY.md §8(d) CPU baseline (1)): initialize, bin, and the first
merges, with the merged occurrences per merge.  Baseline only: the reference never
runs on the GPU box.  Writes profiles/reference_cpu_timing.json.

Usage:  python tools/ref_timing.py [n_chains ...]      (default 200 500)
"""
from __future__ import annotations

import json
import os
import subprocess
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
MERGES = 10


def one(n_chains: int) -> dict:
    sys.path.insert(0, os.path.join(REPO, "pt-bpe_amd"))
    sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
    import numpy as np
    import make_golden
    from geobpe import synth

    make_golden._stub_optional_deps()
    sys.path.insert(0, "/root/reference")
    import foldingdiff.bpe as B
    from foldingdiff.tokenizer import Tokenizer

    B.BPE.visualize = lambda self, key, path: None
    # the first n_chains chains of the C3 corpus (seed 0, U{40..560})
    lengths = synth.make_lengths(100_000, 40, 560, seed=0)[:n_chains]
    corpus = synth.make_corpus(lengths, seed=0)
    structs = []
    for i, row in enumerate(synth.corpus_rows(corpus)):
        s = Tokenizer.init_structure(len(row["phi"]))
        for c in synth.COLUMNS:
            s["angles"][c] = row[c].astype(np.float64)
        s["fname"] = f"synthetic_{i}"
        structs.append(s)
    t0 = time.time()
    bpe = B.BPE(structs, bins={1: 5}, bin_strategy="histogram", save_dir=tempfile.mkdtemp(prefix="geobpe_rt_"),
                rmsd_partition_min_size=float("inf"), res_init=True, std_bonds=True, seed=0)
    bpe.initialize()
    t1 = time.time()
    bpe.bin()
    t2 = time.time()
    steps = []
    for _ in range(MERGES):
        (_, negc, _key), _ = bpe._priority_dict.peekitem(0)
        a = time.time()
        bpe.step()
        steps.append({"count": -negc, "seconds": round(time.time() - a, 3)})
    occ = sum(s["count"] for s in steps)
    sec = sum(s["seconds"] for s in steps)
    return {"chains": n_chains, "residues": int(corpus["row_off"][-1]), "initialize_s": round(t1 - t0, 2),
            "bin_s": round(t2 - t1, 2), "merges": steps, "ms_per_merged_occurrence": round(1000 * sec / occ, 3),
            "merges_per_s": round(MERGES / sec, 4)}


def main(argv):
    if len(argv) == 2 and argv[0] == "--one":
        print("RESULT " + json.dumps(one(int(argv[1]))))
        return
    sizes = [int(x) for x in argv] or [200, 500]
    env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1", MPLBACKEND="Agg", SLURM_CPUS_PER_TASK="0")
    res = []
    for n in sizes:
        r = subprocess.run([sys.executable, "-W", "ignore", __file__, "--one", str(n)], env=env, check=True,
                           stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, text=True, stdin=subprocess.DEVNULL)
        res.append(json.loads([x for x in r.stdout.splitlines() if x.startswith("RESULT ")][-1][7:]))
        print(res[-1], flush=True)
    out = {"generator": "tools/ref_timing.py (reference: /root/reference foldingdiff/bpe.py, this container)",
           "cpus": os.cpu_count(), "corpus": "first n chains of the C3 corpus (seed 0)", "merges_timed": MERGES,
           "runs": res}
    with open(os.path.join(REPO, "profiles", "reference_cpu_timing.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main(sys.argv[1:])
