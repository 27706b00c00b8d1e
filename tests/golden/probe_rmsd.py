"""Probe the REFERENCE's RMSD-partitioned mode in this container.

Runs `foldingdiff.bpe.BPE` with a finite `rmsd_partition_min_size` on a tiny synthetic
corpus and records what initialize() / bin() / step() do: which settings run, which
raise, and the first merges.  Output: tests/golden/rmsd_mode_probe.json (data only).

Usage: python tests/golden/probe_rmsd.py
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

CASES = {
    # name: (p_min_size, num_partitions, max_num_strucs, super_res, merges)
    "p4": (4, {2: 2, 3: 3, 5: 2, 8: 1}, 40, False, 3),
    "p3": (3, {2: 2, 3: 3, 5: 2, 8: 1}, 40, False, 6),
    "p3_super": (3, {2: 2, 3: 3, 5: 2, 8: 1}, 40, True, 6),
    "p0": (0, {2: 2, 3: 3, 5: 2, 8: 1}, 40, False, 6),
    # multi-grid schedules in the RMSD mode (the scoped mode's step() goes stale with them)
    "p0_multigrid": (0, {2: 2, 3: 3, 5: 2, 8: 1}, 40, False, 12, {1: 5, 6: 3, 9: 4}),
    "p0_super_multigrid": (0, {2: 2, 3: 3, 5: 2, 8: 1}, 40, True, 12, {1: 5, 6: 3, 9: 4}),
    "p3_super_multigrid": (3, {2: 2, 3: 3, 5: 2, 8: 1}, 40, True, 12, {1: 4, 7: 6}),
    # free bond lengths (--free-bonds true, the README runs)
    "p0_super_freebonds": (0, {2: 2, 3: 3, 5: 2, 8: 1}, 40, True, 12, {1: 5}, False),
    "p3_freebonds": (3, {2: 2, 3: 3, 5: 2, 8: 1}, 40, False, 12, {1: 5}, False),
}


def run_case(name):
    import numpy as np
    from geobpe import synth
    from make_golden import _stub_optional_deps

    p, nump, maxs, sup, merges = CASES[name][:5]
    bins = CASES[name][5] if len(CASES[name]) > 5 else {1: 5}
    std = CASES[name][6] if len(CASES[name]) > 6 else True
    lengths = synth.make_lengths(8, 20, 40, seed=11)
    corpus = synth.make_corpus(lengths, seed=11)
    _stub_optional_deps()
    sys.path.insert(0, "/root/reference")
    import foldingdiff.bpe as B
    from foldingdiff.tokenizer import Tokenizer

    B.BPE.visualize = lambda self, key, path: None
    Tokenizer.visualize_bonds = lambda self, *a, **k: None
    structs = []
    for i, row in enumerate(synth.corpus_rows(corpus)):
        s = Tokenizer.init_structure(len(row["phi"]))
        for c in synth.COLUMNS:
            s["angles"][c] = row[c].astype(np.float64)
        s["fname"] = f"synthetic_{i}"
        structs.append(s)
    out = {"case": name, "p_min_size": p, "num_partitions": {str(k): v for k, v in nump.items()}, "max_num_strucs": maxs,
           "rmsd_super_res": sup, "events": []}
    try:
        bpe = B.BPE(structs, bins=dict(bins), save_dir=tempfile.mkdtemp(prefix="geobpe_rmsd_probe_"),
                    rmsd_partition_min_size=p, rmsd_super_res=sup, num_partitions=nump,
                    max_num_strucs=maxs, res_init=True, std_bonds=std, seed=0)
        bpe.initialize()
        out["events"].append(["initialize", "ok", len(bpe._tokens), [str(k) for k in list(bpe._tokens)[:12]]])
        bpe.bin()
        out["events"].append(["bin", "ok", len(bpe._priority_dict)])
        for _ in range(merges):
            top = bpe._priority_dict.peekitem(0)[0]
            bpe.step()
            out["events"].append(["step", "ok", str(top[0]), int(top[1]), top[2][:160],
                                  len(bpe._tokens), bpe._step])
    except BaseException as e:  # noqa: BLE001 - the probe records whatever the reference raises
        out["events"].append(["raised", type(e).__name__, str(e)[:300],
                              traceback.format_exc().splitlines()[-6:]])
    return out


def main():
    if len(sys.argv) == 3 and sys.argv[1] == "--one":  # noqa: SIM102
        print("JSON" + json.dumps(run_case(sys.argv[2])))
        return
    env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1", MPLBACKEND="Agg", SLURM_CPUS_PER_TASK="2",
               PYTHONBREAKPOINT="0")
    res = []
    for name in (sys.argv[1:] or CASES):
        r = subprocess.run([sys.executable, "-W", "ignore", __file__, "--one", name], env=env,
                           stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, text=True, timeout=900)
        line = [ln for ln in r.stdout.splitlines() if ln.startswith("JSON")]
        res.append(json.loads(line[-1][4:]) if line else {"case": name, "rc": r.returncode})
        print(json.dumps(res[-1])[:1500], flush=True)
    with open(os.path.join(HERE, "rmsd_mode_probe.json"), "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
