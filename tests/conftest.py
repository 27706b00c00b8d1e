import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "pt-bpe_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


def golden_names():
    # rm_* (tests/test_rmsd_mode.py), gl_* (tests/test_glue.py) and recover_ref (tests/test_recover.py)
    # have layouts of their own
    return sorted(f[:-5] for f in os.listdir(GOLDEN)
                  if f.endswith(".json") and not f.startswith(("rm_", "gl_", "recover_"))
                  and os.path.exists(os.path.join(GOLDEN, f[:-5] + ".npz")))


def pickle_golden_names():
    return sorted(f[:-9] for f in os.listdir(GOLDEN) if f.endswith(".pkl.json"))


def load_golden(name):
    import json

    import numpy as np
    with open(os.path.join(GOLDEN, name + ".json")) as f:
        meta = json.load(f)
    with np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False) as z:
        arrs = {k: z[k] for k in z.files}
    corpus = {k: arrs[k] for k in ["0C:1N", "N:CA", "CA:C", "phi", "psi", "omega", "tau", "CA:C:1N",
                                    "C:1N:1CA", "row_off"]}
    return meta, corpus, arrs


@pytest.fixture(scope="session")
def oracle_lib():
    import oracle
    oracle.build()
    return oracle
