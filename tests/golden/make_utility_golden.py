"""Golden vectors for get_codebook_utility (foldingdiff/plotting.py:78-95): the
reference function itself, run in the build container on the encoded ids of the
reference-made fixtures (tests/golden/*.npz 'ids', vocab size from the .json).
Writes tests/golden/codebook_utility.json.  The reference does not travel: only the
numbers are committed.  Recipe: python tests/golden/make_utility_golden.py"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "..", "..", "pt-bpe_amd"))

FIXTURES = ["g300x60-200_b5", "g80x40-160_b7_rep", "g40x40-120_b12", "c1_pdb12_b5", "g25x1-12_b3_short"]


def main():
    import numpy as np
    import torch
    from make_golden import _stub_optional_deps
    _stub_optional_deps()
    sys.path.insert(0, "/root/reference")
    from foldingdiff.plotting import get_codebook_utility
    out = {}
    for name in FIXTURES:
        meta = json.load(open(os.path.join(HERE, name + ".json")))
        ids = np.load(os.path.join(HERE, name + ".npz"))["ids"].astype(np.int64)
        u = get_codebook_utility(torch.as_tensor(ids), meta["vocab_size"])
        out[name] = {"vocab_size": meta["vocab_size"], "n_ids": int(len(ids)), "utility": u}
    # small hand cases: unused ids, one id, every id once
    for tag, ids, v in (("tiny_unused", [0, 0, 1, 3], 4), ("single", [5] * 7, 9), ("uniform", list(range(16)), 16)):
        out[tag] = {"vocab_size": v, "ids": ids, "utility": get_codebook_utility(torch.as_tensor(ids), v)}
    json.dump(out, open(os.path.join(HERE, "codebook_utility.json"), "w"), indent=1, sort_keys=True)
    print(json.dumps(out, indent=1)[:800])


if __name__ == "__main__":
    main()
