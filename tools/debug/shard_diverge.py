"""Debug: find the first step where the replicated key counts of a
VirtualCluster diverge between ranks."""
import ctypes
import sys

import numpy as np

sys.path.insert(0, "pt-bpe_amd")
sys.path.insert(0, "tests")
sys.path.insert(0, ".")
from conftest import load_golden  # noqa: E402
from geobpe.dist import VirtualCluster  # noqa: E402
from geobpe import _native  # noqa: E402


def counts(e):
    # read the dense counts + key strings of one rank
    L = _native.lib()
    U = e.num_keys
    out = {}
    for d in range(U):
        k = e.key_json(d)
        out.setdefault(k, 0)
    return U


name = sys.argv[1] if len(sys.argv) > 1 else "g25x1-12_b3_short"
world = int(sys.argv[2]) if len(sys.argv) > 2 else 2
meta, corpus, arrs = load_golden(name)
vc = VirtualCluster(corpus, meta["bins"]["1"], world=world).initialize()
vc.bin()
import torch  # noqa: E402


def dump(e):
    L = _native.lib()
    U = e.num_keys
    # copy count array through a debug path: key_json for each key + the per-key count
    # via the C struct (count array pointer) is not exported; use recount instead
    res = {}
    for d in range(U):
        res[d] = e.key_json(d)
    return res


for step in range(len(meta["merges"])):
    sel = []
    for e in vc.engines:
        nid, cnt = ctypes.c_int32(0), ctypes.c_int32(0)
        e._chk(_native.lib().geobpe_step_select(e._ctx, ctypes.byref(nid), ctypes.byref(cnt)))
        sel.append((nid.value, cnt.value, e.L.geobpe_num_keys(e._ctx)))
    print(step, sel, meta["merges"][step][1], flush=True)
    if len(set((a, b) for a, b, _ in sel)) != 1:
        print("DIVERGED at step", step)
        break
    for e in vc.engines:
        nm = ctypes.c_int64(0)
        e._chk(_native.lib().geobpe_step_apply(e._ctx, ctypes.byref(nm)))
    vc._exchange()
