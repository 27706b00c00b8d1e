"""Golden vectors for the structure side of the object API, made by running the REFERENCE in
this container (only the outputs travel):

  Tokenizer.compute_coords()                 tokenizer.py:347-363 (NeRF of the chain's
                                             current geometry; orig=True: the input's)
  BPE.recover_structure(recover(dequantize(quantize(t))), ...)   bpe.py:986-1051
                                             (bin/train.py:715-716)

for the first three chains of a scoped-mode fixture (g40x50_b5, 60 merges) and an
RMSD-mode fixture (rm_p0_super, 25 step() calls).  Output: tests/golden/recover_ref.npz
(coordinates, the recovered structures' 9 columns) + recover_ref.json (bond_to_token of
the recovered tokenizers).

Usage: python tests/golden/make_recover_golden.py
"""
from __future__ import annotations

import json
import os
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "pt-bpe_amd"))
sys.path.insert(0, HERE)
COLS = ["0C:1N", "N:CA", "CA:C", "phi", "psi", "omega", "tau", "CA:C:1N", "C:1N:1CA"]
# name: (fixture, step() calls, kwargs)
CASES = {
    "scoped": ("g40x50_b5", 60, dict(rmsd_partition_min_size=float("inf"))),
    "rmsd": ("rm_p0_super", 25, None),
}


def run():
    import numpy as np
    from geobpe import synth
    from make_golden import _stub_optional_deps
    _stub_optional_deps()
    sys.path.insert(0, "/root/reference")
    import foldingdiff.bpe as RB
    from foldingdiff.tokenizer import Tokenizer
    RB.BPE.visualize = lambda self, key, path: None
    Tokenizer.visualize_bonds = lambda self, *a, **k: None
    arrays, meta = {}, {"generator": "tests/golden/make_recover_golden.py (reference: /root/reference "
                                     "foldingdiff/bpe.py, tokenizer.py)"}
    for case, (fx, calls, kw) in CASES.items():
        with open(os.path.join(HERE, fx + ".json")) as f:
            m = json.load(f)
        with np.load(os.path.join(HERE, fx + ".npz"), allow_pickle=False) as z:
            corpus = {k: z[k] for k in COLS + ["row_off"]}
        structs = []
        for i, row in enumerate(synth.corpus_rows(corpus)):
            s = Tokenizer.init_structure(len(row["phi"]))
            for c in COLS:
                s["angles"][c] = row[c].astype(np.float64)
            s["fname"] = f"synthetic_{i}"
            structs.append(s)
        if kw is None:
            kw = dict(rmsd_partition_min_size=m["rmsd_partition_min_size"], rmsd_super_res=m["rmsd_super_res"],
                      num_partitions={int(a): b for a, b in m["num_partitions"].items()},
                      max_num_strucs=m["max_num_strucs"])
        bpe = RB.BPE(structs, bins={int(a): b for a, b in m["bins"].items()}, save_dir=tempfile.mkdtemp(),
                     res_init=True, std_bonds=True, seed=0, **kw)
        bpe.initialize()
        bpe.bin()
        for _ in range(calls):
            bpe.step()
        meta[case] = {"fixture": fx, "calls": calls, "btt": []}
        for i in range(3):
            t = bpe.tokenizers[i]
            arrays[f"{case}{i}_coords"] = np.asarray(t.compute_coords(), dtype=np.float64)
            arrays[f"{case}{i}_coords_orig"] = np.asarray(t.compute_coords(orig=True), dtype=np.float64)
            dq = bpe.dequantize(bpe.quantize(t))
            t2 = bpe.recover_structure(bpe.recover(dq), dq)
            for c in COLS:
                arrays[f"{case}{i}_rec_{c}"] = np.array([float(x) for x in t2.angles_and_dists[c]])
            arrays[f"{case}{i}_rec_coords"] = np.asarray(t2.compute_coords(), dtype=np.float64)
            meta[case]["btt"].append([[int(s0), list(v[1]) if isinstance(v[1], tuple) else int(v[1]), int(v[2])]
                                      for s0, v in t2.bond_to_token.items()])
    np.savez_compressed(os.path.join(HERE, "recover_ref.npz"), **arrays)
    with open(os.path.join(HERE, "recover_ref.json"), "w") as f:
        json.dump(meta, f)
    print("recover_ref: ok", flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--run":
        run()
    else:
        env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1", MPLBACKEND="Agg", SLURM_CPUS_PER_TASK="2",
                   PYTHONBREAKPOINT="0")
        r = subprocess.run([sys.executable, "-W", "ignore", __file__, "--run"], env=env,
                           stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
        print([ln for ln in r.stdout.splitlines() if ln.startswith("recover_ref")] or r.stderr[-2000:])
