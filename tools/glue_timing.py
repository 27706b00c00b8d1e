"""Time glue optimisation (glue_opt_all): this build vs the reference.

  python tools/glue_timing.py geobpe    [N LO HI]   (GPU box: RmsdBPE.glue_opt_all, one device launch)
  python tools/glue_timing.py reference [N LO HI]   (build container only: foldingdiff, worker pools)

Both run the same synthetic corpus (geobpe.synth, seed 31), bins={1: 5}, p = 0,
num_partitions={2: 2, 3: 5, 5: 2, 8: 1}, max_num_strucs=500, res_init, std_bonds, seed 0,
glue_opt=True (method "all", prior 0), and print one JSON line: initialize seconds and
glue_opt_all seconds (the reference: SLURM_CPUS_PER_TASK = 8 worker processes, this
container's CPUs; torch single-threaded per worker as _opt_glue_worker sets it).
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
sys.path.insert(0, os.path.join(REPO, "pt-bpe_amd"))
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
NUM_P = {2: 2, 3: 5, 5: 2, 8: 1}


def corpus_of(n, lo, hi):
    from geobpe import synth
    return synth.make_corpus(synth.make_lengths(n, lo, hi, seed=31), seed=31)


def run_geobpe(n, lo, hi):
    import torch  # noqa: F401  (HIP runtime shared with torch)
    from geobpe import glue
    from geobpe.bpe import BPE
    corpus = corpus_of(n, lo, hi)
    kern = [0.0, 0]
    f = glue.optimize_chains

    def timed(*a, **k):
        t0 = time.perf_counter()
        r = f(*a, **k)
        kern[0] += time.perf_counter() - t0
        kern[1] += 1
        return r
    glue.optimize_chains = timed
    bpe = BPE(corpus, bins={1: 5}, res_init=True, rmsd_partition_min_size=0, num_partitions=dict(NUM_P),
              max_num_strucs=500, glue_opt=True, glue_opt_method="all", seed=0)
    t0 = time.perf_counter()
    bpe.initialize()
    t1 = time.perf_counter()
    bpe.glue_opt_all()
    t2 = time.perf_counter()
    return {"impl": "geobpe (RmsdBPE.glue_opt_all, one geobpe_glue_opt launch)", "chains": n,
            "residues": int(corpus["row_off"][-1]), "initialize_s": t1 - t0, "glue_opt_all_s": t2 - t1,
            "glue_launch_s": kern[0], "launches": kern[1]}


def run_reference(n, lo, hi):
    from make_golden import _stub_optional_deps
    import numpy as np
    _stub_optional_deps()
    sys.path.insert(0, "/root/reference")
    import foldingdiff.bpe as RB
    from foldingdiff.tokenizer import Tokenizer
    from geobpe import synth
    corpus = corpus_of(n, lo, hi)
    structs = []
    for i, row in enumerate(synth.corpus_rows(corpus)):
        s = Tokenizer.init_structure(len(row["phi"]))
        for c in row:
            s["angles"][c] = row[c].astype(np.float64)
        s["fname"] = f"synthetic_{i}"
        structs.append(s)
    bpe = RB.BPE(structs, bins={1: 5}, save_dir=tempfile.mkdtemp(prefix="geobpe_glue_timing_"),
                 rmsd_partition_min_size=0, num_partitions=dict(NUM_P), max_num_strucs=500, res_init=True,
                 std_bonds=True, glue_opt=True, glue_opt_method="all", seed=0)
    t0 = time.perf_counter()
    bpe.initialize()
    t1 = time.perf_counter()
    bpe.glue_opt_all()
    t2 = time.perf_counter()
    return {"impl": "reference (foldingdiff.bpe.BPE.glue_opt_all, 8 worker processes)", "chains": n,
            "residues": int(corpus["row_off"][-1]), "initialize_s": t1 - t0, "glue_opt_all_s": t2 - t1,
            "cpus": os.cpu_count()}


def main(argv):
    which = argv[0]
    n, lo, hi = (int(x) for x in (argv[1:4] if len(argv) >= 4 else (64, 60, 300)))
    if which == "reference" and os.environ.get("SLURM_CPUS_PER_TASK") is None:
        env = dict(os.environ, SLURM_CPUS_PER_TASK=str(os.cpu_count()), PYTHONBREAKPOINT="0", MPLBACKEND="Agg")
        r = subprocess.run([sys.executable, "-W", "ignore", __file__] + argv, env=env, stdout=subprocess.PIPE, text=True)
        print(r.stdout.strip().splitlines()[-1])
        return
    out = run_geobpe(n, lo, hi) if which == "geobpe" else run_reference(n, lo, hi)
    print(json.dumps(out))


if __name__ == "__main__":
    main(sys.argv[1:])
