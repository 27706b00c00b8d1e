"""Stress the sharded (VirtualCluster) path on the small golden fixtures; after
every exchange compare the replicated key counts of all ranks."""
import sys

sys.path.insert(0, "pt-bpe_amd")
sys.path.insert(0, "tests")
sys.path.insert(0, ".")
from conftest import load_golden  # noqa: E402
from geobpe.dist import VirtualCluster  # noqa: E402
from geobpe.engine import GeoBPEEngine  # noqa: E402

bad = 0
for rep in range(int(sys.argv[1]) if len(sys.argv) > 1 else 10):
    # churn device memory like the test suite does
    for name in ["g40x50_b5", "g300x60-200_b5"]:
        meta, corpus, _ = load_golden(name)
        e = GeoBPEEngine(corpus, meta["bins"]["1"]).initialize()
        e.bin()
        e.run(20)
        e.close()
    for name, world in [("g25x1-12_b3_short", 2), ("g25x1-12_b3_short", 3), ("g60x20-90_b5_rep", 3)]:
        meta, corpus, _ = load_golden(name)
        vc = VirtualCluster(corpus, meta["bins"]["1"], world=world).initialize()
        vc.bin()
        for step in range(len(meta["merges"]) + 1):
            try:
                cs = [e.key_counts() for e in vc.engines]
            except IndexError as ex:
                import ctypes, numpy as np
                from geobpe import _native
                d = int(str(ex))
                for r, e in enumerate(vc.engines):
                    o = np.zeros(9, dtype=np.int64)
                    _native.lib().geobpe_debug_key(e._ctx, d, o.ctypes.data_as(ctypes.c_void_p))
                    print("rank", r, "key", d, "idL,g,idR,len,count,U,Kdev,Khost,h1 =", o.tolist(), flush=True)
                print("at rep", rep, name, world, "step", step, flush=True)
                raise
            if any(c != cs[0] for c in cs[1:]):
                bad += 1
                diff = {k: [c.get(k) for c in cs] for k in set().union(*cs) if len({c.get(k) for c in cs}) > 1}
                print(f"rep {rep} {name} w{world} step {step}: {len(diff)} keys differ, e.g.", list(diff.items())[:3],
                      flush=True)
                break
            if step == len(meta["merges"]):
                break
            try:
                vc.step()
            except Exception as ex:
                print("step error", rep, name, world, step, ex, flush=True)
                bad += 1
                break
        vc.close()
print("bad", bad)
