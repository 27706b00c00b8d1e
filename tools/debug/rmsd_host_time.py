"""Host time of the RMSD-partitioned mode's step() (RmsdBPE) on the CPU, without a profiler:
the device batches (NeRF, Kabsch RMSD, thresholds) replaced by batched numpy stand-ins (not
the oracle's per-pair loops: only their time is subtracted, their results steer k-medoids),
and the host pieces of a step timed one by one by wrapping them.  The number to compare with
the box's rmsd_timing_*.json is "host ms per step".

  python tools/debug/rmsd_host_time.py [N LO HI STEPS] [--device | --fake] [--cprofile] [--sample] [--warm=5]   (default 2000 40 120 50)

--device (GPU box): the real device batches, timed and subtracted the same way; the CPU
stand-ins evict the host state from the caches, so only this mode gives the box's host time."""
import os
import sys
import time
from collections import defaultdict

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "pt-bpe_amd"))
sys.path.insert(0, ROOT)

import oracle.prologue as prologue  # noqa: E402
import oracle.rmsd as orm  # noqa: E402
from geobpe import rmsd, rmsd_bpe, synth  # noqa: E402
from geobpe.bpe import BPE  # noqa: E402

DEVICE = "--device" in sys.argv
CPROF = "--cprofile" in sys.argv  # (then the top functions by own time, after the timings)
WARM = int(next((a.split("=")[1] for a in sys.argv if a.startswith("--warm=")), 5))  # (untimed steps first;
#  tools/rmsd_mode_timing.py, the number DESIGN quotes, times steps 1..50: --warm=0)
argv = [a for a in sys.argv[1:] if not a.startswith("--")]
n, lo, hi, steps = (int(x) for x in (argv[:4] if len(argv) >= 4 else (2000, 40, 120, 50)))
stand = [0.0]
parts = defaultdict(float)


def kabsch(P, Q):
    """rmsd of P[i] against Q[i] (float64 (n, a, 3) each), batched"""
    P = P - P.mean(axis=1, keepdims=True)
    Q = Q - Q.mean(axis=1, keepdims=True)
    H = np.einsum("nai,naj->nij", Q, P)
    U, _, Vt = np.linalg.svd(H)
    d = np.sign(np.linalg.det(U @ Vt))
    Vt[:, 2, :] *= d[:, None]
    R = U @ Vt
    res = P - Q @ R
    return np.sqrt(np.mean(np.sum(res * res, axis=2), axis=1))


def rmsd_matrix(S):
    S = np.asarray(S, dtype=np.float64)
    N = len(S)
    i, j = np.triu_indices(N)
    D = np.empty((N, N), dtype=np.float32)
    for a in range(0, len(i), 1 << 16):
        v = kabsch(S[i[a:a + (1 << 16)]], S[j[a:a + (1 << 16)]])
        D[i[a:a + (1 << 16)], j[a:a + (1 << 16)]] = v
        D[j[a:a + (1 << 16)], i[a:a + (1 << 16)]] = v
    return D


def rmsd_cross(A, B):
    A, B = np.asarray(A, dtype=np.float64), np.asarray(B, dtype=np.float64)
    ii, jj = np.meshgrid(np.arange(len(A)), np.arange(len(B)), indexing="ij")
    return kabsch(A[ii.ravel()], B[jj.ravel()]).reshape(len(A), len(B))


def timed(f, acc=None):
    def g(*a, **k):
        t0 = time.perf_counter()
        r = f(*a, **k)
        dt = time.perf_counter() - t0
        if acc is None:
            stand[0] += dt
        else:
            parts[acc] += dt
        return r
    return g


FAKE = "--fake" in sys.argv  # (CPU: cheap deterministic stand-ins -- random distances, zero atoms
#  -- so the host work is measured without numpy evicting it from the caches; the merges then
#  differ from the real ones, so only A/Bs of host code on the same workload are meaningful)
if FAKE:
    def fake_run(a, b, symmetric, device):
        nb = a.shape[0] if symmetric else b.shape[0]
        return np.random.default_rng(7 * a.shape[0] + nb).random((a.shape[0], nb)) * 3
    rmsd._run = timed(fake_run)
    rmsd.nerf_atoms = timed(lambda off, packed, device=0: np.zeros((max(int(off[-1]), 1) * 3, 3)))
    rmsd_bpe.RmsdBPE._grid_thresholds = lambda self: {s: prologue.thresholds(self._corpus, b)
                                                      for s, b in self.bins.items()}
elif DEVICE:
    import torch  # noqa: F401  (HIP runtime shared with torch)
    for nm in ("_run", "nerf_atoms"):  # (the leaves: every device batch goes through one)
        setattr(rmsd, nm, timed(getattr(rmsd, nm)))
else:
    rmsd.geo_coords = timed(lambda geos, device=0: [orm.nerf(g) for g in geos])
    rmsd.nerf_packed = timed(lambda off, packed, device=0: orm.nerf_packed(off, packed))
    rmsd.nerf_atoms = timed(lambda off, packed, device=0: orm.nerf_atoms(off, packed))
    rmsd.rmsd_matrix = timed(lambda S, device=0: rmsd_matrix(S))
    rmsd.rmsd_cross = timed(lambda A, B, device=0: rmsd_cross(A, B))
    rmsd_bpe.RmsdBPE._grid_thresholds = lambda self: {s: prologue.thresholds(self._corpus, b)
                                                      for s, b in self.bins.items()}

def _sampler():
    import importlib.util
    import subprocess
    import sysconfig
    src = os.path.join(ROOT, "tools", "debug", "sampler.c")
    so = os.path.join("/tmp", "_sampler.so")
    subprocess.run(["gcc", "-O2", "-shared", "-fPIC", f"-I{sysconfig.get_paths()['include']}", src, "-o", so], check=True)
    spec = importlib.util.spec_from_file_location("_sampler", so)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _resolve(pcs, top=40):
    """(library, symbol) counts of the sampled pcs; our _rmsdkey.so by source line (addr2line)"""
    import ctypes
    import subprocess
    from collections import Counter

    class DlInfo(ctypes.Structure):
        _fields_ = [("fname", ctypes.c_char_p), ("fbase", ctypes.c_void_p), ("sname", ctypes.c_char_p),
                    ("saddr", ctypes.c_void_p)]
    dladdr = ctypes.CDLL(None).dladdr
    dladdr.argtypes = [ctypes.c_void_p, ctypes.POINTER(DlInfo)]
    by_sym, ours = Counter(), Counter()
    for pc, c in Counter(pcs).items():
        d = DlInfo()
        if not dladdr(ctypes.c_void_p(pc), ctypes.byref(d)):
            by_sym[("?", "?")] += c
            continue
        lib = os.path.basename((d.fname or b"?").decode())
        if "_rmsdkey" in lib:
            ours[(d.fname.decode(), pc - d.fbase)] += c
            by_sym[(lib, "(by line below)")] += c
        else:
            by_sym[(lib, (d.sname or b"?").decode())] += c
    n = max(len(pcs), 1)
    print(f"  {len(pcs)} samples")
    for (lib, sym), c in by_sym.most_common(top):
        print(f"  {100 * c / n:5.1f}%  {lib:28s} {sym}")
    if ours:
        lines = Counter()
        for (f, off), c in ours.items():
            r = subprocess.run(["addr2line", "-f", "-s", "-e", f, hex(off)], capture_output=True, text=True).stdout.split()
            lines[" ".join(r[:2]) if r else hex(off)] += c
        for ln, c in lines.most_common(top):
            print(f"  {100 * c / n:5.1f}%  rmsdkey {ln}")


corpus = synth.make_corpus(synth.make_lengths(n, lo, hi, seed=31), seed=31)
if "--readme" in sys.argv:  # (bench.py --config rmsd's setting, README.md:45, without the glue optimisation)
    bpe = BPE(corpus, bins={1: 50}, bin_strategy="histogram", res_init=True, std_bonds=False,
              rmsd_partition_min_size=0, rmsd_super_res=True, num_partitions={2: 2, 3: 5, 5: 1, 6: 2, 8: 1},
              max_num_strucs=500, seed=0)
else:
    bpe = BPE(corpus, bins={1: 5}, res_init=True, rmsd_partition_min_size=0, rmsd_super_res=True,
              num_partitions={2: 2, 3: 5, 5: 2, 8: 1}, max_num_strucs=500, seed=0)
bpe.initialize()
bpe.bin()
bpe.run(WARM)
# the host pieces (their stand-in time inside is in stand, subtracted from each below)
K = rmsd_bpe._KEYC
wrapped = {}
for nm in ("_partition", "_assign", "_span_coords", "_struc_coords"):
    wrapped[nm] = getattr(rmsd_bpe.RmsdBPE, nm)


class KeyC:
    def __getattr__(self, a):
        return getattr(K, a)

    def merge(self, *a):
        t0 = time.perf_counter()
        r = K.merge(*a)
        parts["C merge"] += time.perf_counter() - t0
        return r

    def prio(self, *a):
        t0 = time.perf_counter()
        r = K.prio(*a)
        parts["C prio"] += time.perf_counter() - t0
        return r


rmsd_bpe._KEYC = KeyC()
for nm, f in wrapped.items():
    def mk(f, nm):
        def g(self, *a, **k):
            s0 = stand[0]
            t0 = time.perf_counter()
            r = f(self, *a, **k)
            parts[nm] += time.perf_counter() - t0 - (stand[0] - s0)
            return r
        return g
    setattr(rmsd_bpe.RmsdBPE, nm, mk(f, nm))
s0 = stand[0]
m0 = len(bpe._merge_log)
parts.clear()
SAMPLE = "--sample" in sys.argv  # (SIGPROF samples of the steps: tools/debug/sampler.c, built on use)
if SAMPLE:
    smp = _sampler()
    smp.start(100)
if CPROF:
    import cProfile
    import pstats
    prof = cProfile.Profile()
    prof.enable()
t0 = time.perf_counter()
done = bpe.run(steps)
t = time.perf_counter() - t0
if CPROF:
    prof.disable()
if SAMPLE:
    pcs = smp.stop()
host = t - (stand[0] - s0)
print(f"{done} steps: {1000 * t / done:.2f} ms per step, of which stand-ins {1000 * (stand[0] - s0) / done:.2f} ms; "
      f"host {1000 * host / done:.2f} ms per step")
nested = {"_assign", "_span_coords", "_struc_coords"}  # (inside _partition or the recurring path)
for k, v in sorted(parts.items(), key=lambda x: -x[1]):
    print(f"  {k:16s} {1000 * v / done:7.3f} ms/step")
print(f"  {'rest (Python)':16s} {1000 * (host - sum(v for k, v in parts.items() if k not in nested and k != '_partition') - parts['_partition']) / done:7.3f} ms/step")
print("  first merges (count, ms):", [(m[1], round(1000 * x, 2)) for m, x in
                                      list(zip(bpe._merge_log, bpe._times))[m0:m0 + 12]])
if hasattr(K, "prof"):
    labels = ["removals", "token rewrite", "set_geo", "new keys", "new-key sets", "bin set_geo", "build_key", "key str"]
    for lab, (ns, cnt) in zip(labels, K.prof()):
        print(f"  C {lab:14s} {ns / 1e6 / (done + WARM):7.3f} ms/step ({cnt} calls)")
if CPROF:
    pstats.Stats(prof).sort_stats("tottime").print_stats(30)
if SAMPLE:
    _resolve(pcs)
