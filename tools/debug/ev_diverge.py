"""Where does the device merge list leave the oracle's on the merge-event corpus
(with / without event recording)?"""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "pt-bpe_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import numpy as np
import torch  # noqa
from geobpe import synth
from geobpe.engine import GeoBPEEngine
import oracle
lengths = synth.make_lengths(2000, 20, 200, seed=71)
corpus = synth.make_corpus(lengths, seed=71, repeat_frac=0.1)
o = oracle.OracleBPE(corpus, 5).initialize(); o.bin()
for _ in range(300): o.step()
om = list(o.merges)
for ev in (False, True, False):
    for mode in ("run", "step"):
        e = GeoBPEEngine(corpus, 5).initialize(); e.bin()
        if ev: e.record_events(True)
        if mode == "run": e.run(300)
        else:
            for _ in range(300): e.step()
        m = e.merge_keys()
        d = next((i for i in range(min(len(m), len(om))) if m[i] != om[i]), None)
        print("events", ev, mode, "first diff", d, (m[d][1], om[d][1]) if d is not None else "", "verify", e.verify_counts(), flush=True)
        e.close()
