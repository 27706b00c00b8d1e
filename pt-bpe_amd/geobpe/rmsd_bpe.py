"""GeoBPE in the reference's RMSD-partitioned mode.

With a finite ``rmsd_partition_min_size`` (p) the reference's ``BPE`` turns every token of at
least p bonds into a family of k-medoids partitions under Kabsch RMSD:

  reference (foldingdiff/bpe.py)                 here
  _init_res_tokens, res_geo branch  :231-379     RmsdBPE._init_residues / _partition_residues
  compute_geo_key (pt1 / pt2 rules) :1192-1299   RmsdBPE._pair_key
  bin                               :1431-1474   RmsdBPE.bin
  rmsd_partition                    :1739-1789   RmsdBPE._partition
  step (RMSD branches, recurring    :1792-2166   RmsdBPE.step / _merge
    keys, the repeat at :2164-2166)
  _compute_assignment(_inner)       :645-657     RmsdBPE._assign (one device batch)
  Tokenizer.compute_coords /        tokenizer.py:347-363, :204-230
    key_coords                                   RmsdBPE._span_coords / _struc_coords

Where the time goes in the reference -- NeRF coordinates and Kabsch RMSD of every
occurrence against every medoid (process pools), and the O(M^2) k-medoids matrix -- runs on
the GPU here as batches: one ``geobpe_nerf`` launch for all occurrences of a key, one
``geobpe_rmsd`` launch for the matrix and one for occurrences x medoids (csrc/rmsd.h).

The bookkeeping around them is host code, because the keys stop being content hashes in
this mode: a partitioned token's interior enters the key as raw floats (the medoid's
geometry) and the junction as bin indices (bpe.py:1247-1296), so the key of a span depends on
where it is split and on which medoid each side was assigned.  The device engine of the
scoped mode (split-invariant 2x61-bit content hashes) does not apply; this class keeps the
reference's dictionaries instead, with the same add/remove sequence per key, so
``list(_geo_dict[key])`` -- the order k-medoids sees the occurrences in -- is the reference's.

Reachable configurations (tests/golden/rmsd_mode_probe.json, rm_p4.json): p <= 3 partitions
the residues at initialize() and every merge; p >= 4 never creates ``_sphere_dict``, so the
first merge of >= p bonds raises AttributeError there, as it does here.  Glue optimisation
(``glue_opt=True``, ``glue_opt_method="all"``, bpe.py:106-135, 192-229, 2027-2071) runs as one
device L-BFGS launch over the chains (geobpe/glue.py, csrc/glue.h).  The "each" method
stops where the reference's does (an AssertionError in initialize(), bpe.py:761).
``rmsd_only`` (bpe.py:1977, 2027) keeps a partitioned merge's own geometry: the medoid's is
not written over it, and no glue is re-optimised.  Free bond lengths
(``std_bonds=False``) run where the reference runs them (p <= 2; p >= 3 raises its KeyError).
"""
from __future__ import annotations

import bisect
import gc
import heapq
import json
import os
import time
from collections import defaultdict

import numpy as np

from . import rmsd as _rmsd
from .synth import COLUMNS

BOND_TYPES = ["N:CA", "CA:C", "0C:1N"]
BOND_ANGLES = ["tau", "CA:C:1N", "C:1N:1CA"]
DIHEDRALS = ["psi", "omega", "phi"]
GLUE = ["omega", "C:1N:1CA", "phi"]                            # bpe.py:383
TWO_PI = 2 * np.pi
# the residue-level partition keys of _sphere_dict (bpe.py:333-338)
# item type -> (position of its first item in a residue, kind: 0 bond, 1 angle, 2 dihedral)
_ITEM = {k: (i, 0) for i, k in enumerate(BOND_TYPES)} | {k: (i, 1) for i, k in enumerate(BOND_ANGLES)} | \
    {k: (i, 2) for i, k in enumerate(DIHEDRALS)}
_ENC = json.JSONEncoder(sort_keys=True)  # json.dumps(geo, sort_keys=True) (bpe.py:1147-1149)
_KEY_ORDER = sorted(_ITEM)  # json key order of the nine item types
_KEY_ORDER_T = tuple(_KEY_ORDER)
_PACK_ORDER = ["N:CA", "CA:C", "tau", "0C:1N", "CA:C:1N", "C:1N:1CA", "psi", "omega", "phi"]  # geobpe_nerf's


def _load_keyc():
    """The C pair-key builder (csrc/rmsdkey.c, built in-tree by geobpe/build.py)."""
    import importlib.util
    import os
    # (GEOBPE_RMSDKEY: another build of the same extension, e.g. tools/asan_host.sh's sanitizer build)
    path = os.environ.get("GEOBPE_RMSDKEY") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "_rmsdkey.so")
    if not os.path.exists(path):
        return None
    spec = importlib.util.spec_from_file_location("_rmsdkey", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


_KEYC = _load_keyc()


class _PrioQueue:
    """The reference's priority SortedDict of (not partitioned, -count, key) entries
    (bpe.py:1431-1474, 2077-2138) as a heap with lazy deletion.  `live` is _key_to_priority
    itself (key -> its current entry); a heap entry whose key no longer maps to that very tuple
    is stale and leaves when it reaches the top.  Keys are unique, so the tuple order the heap
    keeps is the sorted container's order; only [0], len, add, remove and sorted iteration are
    used.  (A SortedList add/remove cost ~2 us each, a third of a 2000-chain step.)"""
    __slots__ = ("heap", "live")

    def __init__(self, live: dict):
        self.live = live
        self.heap = list(live.values())
        heapq.heapify(self.heap)

    def add(self, pr):
        self.live[pr[2]] = pr
        heapq.heappush(self.heap, pr)

    def remove(self, pr):
        if self.live.get(pr[2]) is pr:
            del self.live[pr[2]]

    def _top(self):
        h, live = self.heap, self.live
        while h and live.get(h[0][2]) is not h[0]:
            heapq.heappop(h)
        if len(h) > 2 * len(live) + 4096:  # (stale entries deep in the heap: rebuild)
            self.heap = h = list(live.values())
            heapq.heapify(h)
        if not h:
            raise IndexError("priority queue is empty")
        return h[0]

    def __len__(self):
        return len(self.live)

    def __getitem__(self, i):
        if i == 0:
            return self._top()
        return sorted(self.live.values())[i]

    def __iter__(self):
        return iter(sorted(self.live.values()))
RES_SPHERE_KEY = {3: '{"N:CA": [0], "CA:C": [0], "0C:1N": [0], "tau": [0], "CA:C:1N": [0], "psi": [0]}',
                  2: '{"CA:C": [0], "0C:1N": [0], "CA:C:1N": [0]}'}


_LEFT = {}


def _pk_at(pk, ci, i):
    """The stored key of the pair starting at bond i of chain ci (pk: that chain's list);
    KeyError((ci, i)) when no pair starts there, as the reference's dict lookup raises."""
    k = pk[i] if i < len(pk) else None
    if k is None:
        raise KeyError((ci, i))
    return k


def _get_ind(v, values):
    """BPE.get_ind (bpe.py:1164-1189), with the left edges of each threshold list cached."""
    left = _LEFT.get(id(values))
    if left is None or left[0] is not values:
        left = _LEFT[id(values)] = (values, [a for a, _ in values])
    ind = bisect.bisect_right(left[1], v) - 1
    if ind < 0:
        raise ValueError(f"value {v} is below the first bin range")
    a, b = values[ind]
    if ind == len(values) - 1 and v == b:
        return ind
    if a <= v < b:
        return ind
    raise ValueError(f"value {v} does not fall into any bin")


class _Chain:
    """One chain's internal coordinates (current and original) and segmentation: the state
    of the reference's Tokenizer that this mode reads and writes (tokenizer.py:131-202,
    253-286).  Bond j -> init N:CA / CA:C for j < 2, else column BOND_TYPES[j%3] row
    (j-2)//3; angle a -> init tau for a = 0, else BOND_ANGLES[a%3] row (a-1)//3; dihedral d ->
    DIHEDRALS[d%3] row (d+1)//3.  The init values are shared by both copies (the
    reference's ``orig`` flag only switches the DataFrame)."""

    __slots__ = ("cur", "orig", "init", "n", "token_pos", "btt", "fname", "tokens0", "events")

    def __init__(self, cols: dict, init, fname=None):
        # Python lists: the host bookkeeping reads and writes single values (the
        # reference's object DataFrame cells); numpy scalar indexing is ~5x slower here
        self.cur = {c: [float(v) for v in cols[c]] for c in COLUMNS}
        self.orig = {c: [float(v) for v in cols[c]] for c in COLUMNS}
        self.init = list(init)
        self.n = len(self.cur["phi"])
        self.token_pos = []
        self.btt = {}
        self.fname = fname
        self.tokens0 = []  # Tokenizer.tokens: the initial tokens (step() never updates them, bpe.py:1955-1965)
        self.events = []   # merge tree: (left start, right start, parent value) per merge (data_structures.py:32-60)

    def _angle(self, a, src):
        return self.init[2] if a == 0 else src[BOND_ANGLES[a % 3]][(a - 1) // 3]

    def _dihedral(self, d, src):
        return src[DIHEDRALS[d % 3]][(d + 1) // 3]

    def geo(self, idx, l, orig=False):
        """token_geo(idx, l, orig) (tokenizer.py:169-202).  Same-type items of a span sit
        in consecutive rows of their column, so each type is one slice (bonds 0, 1 and
        angle 0 are the chain's init values, in front of their column's rows)."""
        if idx + l - 1 > 3 * self.n - 1:
            raise ValueError(f"idx+l cannot exceed {3 * self.n - 1}")
        src = self.orig if orig else self.cur
        init = self.init
        out = {}
        for j in range(idx, idx + min(l, 3)):  # bonds: row (j - 2) // 3; j < 2 -> init
            k, cnt = BOND_TYPES[j % 3], len(range(j, idx + l, 3))
            out[k] = [init[j]] + src[k][:cnt - 1] if j < 2 else src[k][(j - 2) // 3:(j - 2) // 3 + cnt]
        for a in range(idx, idx + min(l - 1, 3)):  # angles: row (a - 1) // 3; a = 0 -> init
            k, cnt = BOND_ANGLES[a % 3], len(range(a, idx + l - 1, 3))
            out[k] = [init[2]] + src[k][:cnt - 1] if a == 0 else src[k][(a - 1) // 3:(a - 1) // 3 + cnt]
        for d in range(idx, idx + min(l - 2, 3)):  # dihedrals: row (d + 1) // 3
            k, cnt = DIHEDRALS[d % 3], len(range(d, idx + l - 2, 3))
            out[k] = src[k][(d + 1) // 3:(d + 1) // 3 + cnt]
        return out

    def set_geo(self, idx, l, vals):
        """set_token_geo(idx, l, vals) (tokenizer.py:253-286): values consumed in order.  In C
        (csrc/rmsdkey.c setgeo) when the values fit exactly; otherwise here, which raises the
        reference's error at the same point."""
        if _KEYC is not None and type(vals) is dict and \
                _KEYC.setgeo(tuple(self.cur[k] for k in _KEY_ORDER), self.init, idx, l, vals):
            return
        it = {k: iter(v) for k, v in vals.items()}
        for j in range(idx, idx + l):
            v = next(it[BOND_TYPES[j % 3]])
            if j < 2:
                self.init[j] = v
            else:
                self.cur[BOND_TYPES[j % 3]][(j - 2) // 3] = v
        for j in range(idx, idx + l - 1):
            v = next(it[BOND_ANGLES[j % 3]])
            if j == 0:
                self.init[2] = v
            else:
                self.cur[BOND_ANGLES[j % 3]][(j - 1) // 3] = v
        for j in range(idx, idx + l - 2):
            self.cur[DIHEDRALS[j % 3]][(j + 1) // 3] = next(it[DIHEDRALS[j % 3]])
        for k, rest in it.items():
            if next(rest, None) is not None:
                raise AssertionError(f"set_token_geo: values of {k} left over")

    def tokens(self):
        return list(self.btt.values())

    def glue(self, b):
        """The three glue values after a token ending before bond b (tokenizer.py:384-391)."""
        return (self._dihedral(b - 2, self.cur), self._dihedral(b - 1, self.cur), self._angle(b - 1, self.cur))


def chain_coords(c: "_Chain", index=0, length=float("inf"), orig=False, device: int = 0):
    cols = c.orig if orig else c.cur
    ln = min(length, 3 * c.n - 1 - index)
    return _rmsd.compute_coords(cols, [(index, int(ln))], init=tuple(c.init), device=device)[0]


def init_structure(n: int) -> dict:
    """Tokenizer.init_structure / BPE.init_structure (tokenizer.py:395-417, bpe.py:1005-1027)."""
    import pandas as pd
    angles = {c: [0.0] * n if c in BOND_TYPES else [np.nan] * n for c in COLUMNS}
    idxes = sum([[i, i, i] for i in range(1, n + 1)], [])
    return {"angles": pd.DataFrame(angles), "coords": None, "c_beta": None, "full_idxes": idxes,
            "full_coords": None, "side_chain": None, "aa": None, "fname": None}


def recover_structure(tokens: dict, repl: dict, tokenized, device: int = 0) -> "RmsdTokenizer":
    """BPE.recover_structure (bpe.py:1029-1051): a chain whose rows come from the recovered
    geometry (the init bond / angle of residue 0 dropped, the last row left at the
    init_structure defaults), the raw init triple of a new Tokenizer, and one token per
    MOTIF of ``tokenized`` with its id's bond count."""
    n = len(repl["N:CA"])
    cols = {c: [0.0] * n if c in BOND_TYPES else [np.nan] * n for c in COLUMNS}

    def put(c, lo, hi, vals):
        vals = list(vals)
        rows = list(range(n))[lo:hi]
        if len(vals) != len(rows):
            raise ValueError(f"recover_structure: {c} has {len(vals)} values for {len(rows)} rows")
        for r, v in zip(rows, vals):
            cols[c][r] = float(v)

    put("N:CA", None, -1, repl["N:CA"][1:])
    put("CA:C", None, -1, repl["CA:C"][1:])
    put("0C:1N", None, -1, repl["0C:1N"])
    put("phi", 1, None, repl["phi"])
    put("psi", None, -1, repl["psi"])
    put("omega", None, -1, repl["omega"])
    put("tau", None, -1, repl["tau"][1:])
    put("CA:C:1N", None, -1, repl["CA:C:1N"])
    put("C:1N:1CA", None, -1, repl["C:1N:1CA"])
    c = _Chain(cols, _rmsd.init_geometry())
    cur = 0
    for tok in tokenized:
        if tok[0] == "MOTIF":
            nb = sum(len(tokens[tok[1]].get(k, [])) for k in BOND_TYPES)
            c.btt[cur] = (cur, tok[1], nb)
            c.token_pos.extend([cur] * nb)
            cur += nb
    c.tokens0 = list(c.btt.values())
    return RmsdTokenizer(c, device)


class RmsdTokenizer:
    """Tokenizer view of one chain in the RMSD mode: ``bond_to_token`` with tuple ids
    ``(n, p)``, ``token_pos``, ``tokens``, ``tokenize()`` (tokenizer.py:379-392)."""

    def __init__(self, chain: _Chain, device: int = 0):
        self._c = chain
        self.n = chain.n
        self.fname = chain.fname
        self._device = device

    def compute_coords(self, index=0, length=float("inf"), orig=False):
        """Tokenizer.compute_coords (tokenizer.py:347-363): backbone atoms of bonds
        index..index+length by NeRF of the chain's current (or original) geometry, on the
        device; the init lengths / angle are the chain's current ones in both cases."""
        return chain_coords(self._c, index, length, orig, self._device)

    @property
    def bond_to_token(self):
        return dict(self._c.btt)

    @property
    def token_pos(self):
        return list(self._c.token_pos)

    @property
    def tokens(self):
        return self._c.tokens()

    def token_geo(self, idx, l, orig=False):
        return self._c.geo(idx, l, orig)

    def tokenize(self):
        out = []
        last = 3 * self.n - 1
        for start, tid, length in self._c.btt.values():
            out.append(("MOTIF", tid))
            b = start + length
            if b < last:
                om, ph, cn = self._c.glue(b)
                out.append(("DIHEDRAL", DIHEDRALS[(b - 2) % 3], om))
                out.append(("DIHEDRAL", DIHEDRALS[(b - 1) % 3], ph))
                out.append(("BOND_ANGLE", BOND_ANGLES[(b - 1) % 3], cn))
        return out


class _RmsdGroup:
    """The RMSD mode over several processes (``RmsdBPE(group=...)``): every rank holds the whole
    corpus and the same host state (the bookkeeping is replicated and deterministic), and the
    per-merge assignment batch is split across the ranks.  ``group``: a torch.distributed
    process group, ``True`` for the default one, or an object carrying one as ``.pg``
    (geobpe.dist.TorchGroup)."""

    def __init__(self, group, device: int):
        import torch
        import torch.distributed as dist
        pg = None if group is True else getattr(group, "pg", group)
        self.torch, self.dist, self.pg = torch, dist, pg
        self.rank = dist.get_rank(pg)
        self.world = dist.get_world_size(pg)
        # (NCCL gathers on the GPU this rank's batches run on, not torch's current device)
        self.dev = torch.device("cuda", device) if dist.get_backend(pg) == "nccl" else torch.device("cpu")

    def shared_seed(self):
        """a seed drawn by rank 0 and broadcast: with seed=None (the reference's default) every
        rank's Generator must still make the same draws (k-medoids' picks are replicated state)"""
        box = [int(np.random.SeedSequence().entropy) if self.rank == 0 else None]
        self.dist.broadcast_object_list(box, src=0, group=self.pg)
        return box[0]

    def barrier(self):
        self.dist.barrier(group=self.pg)

    def gather_chunks(self, mine: np.ndarray, n: int) -> np.ndarray:
        """The ranks' contiguous chunks [n * r // world, n * (r + 1) // world) of an int64
        array of n, all-gathered in rank order"""
        torch = self.torch
        w = self.world
        cap = -(-n // w) + 1
        t = torch.full((cap,), -1, dtype=torch.int64)
        t[:len(mine)] = torch.from_numpy(mine)
        t = t.to(self.dev)
        outs = [torch.empty_like(t) for _ in range(w)]
        self.dist.all_gather(outs, t, group=self.pg)
        parts = [outs[r][:n * (r + 1) // w - n * r // w].cpu().numpy() for r in range(w)]
        return np.concatenate(parts)


class RmsdBPE:
    """foldingdiff.bpe.BPE with a finite rmsd_partition_min_size (see the module docstring).
    Constructed by ``geobpe.bpe.BPE(...)`` when the arguments ask for this mode."""

    _py_keys = False  # True: the pair keys in Python (_pair_key_py) instead of csrc/rmsdkey.c
    _no_key_memo = False  # True: rmsdkey.c merge derives every pair key (no memo; A/B and tests)
    _group = None  # _RmsdGroup with a process group (also what a checkpoint-loaded instance has)

    def __init__(self, structures, bins, bin_strategy="histogram", save_dir="./plots/bpe",
                 compute_sec_structs=False, plot_iou_with_sec_structs=False, res_init=False, std_bonds=True,
                 rmsd_partition_min_size=4, rmsd_super_res=False, rmsd_only=False, num_partitions=3,
                 max_num_strucs=500, glue_opt=False, glue_opt_prior=0.0, glue_opt_every=10,
                 glue_opt_method="all", seed=None, device=None, group=None, **_unused):
        from .bpe import ThresholdDict, structures_to_corpus
        if not isinstance(bins, dict) or 1 not in bins:
            raise KeyError("bins must be a dict with key 1 (quantize/capacity need bins[1], bpe.py:896,909,952)")
        if not res_init and not std_bonds:  # (no reference fixture pins it)
            raise NotImplementedError("bond-level init (res_init=False) with free bond lengths is not built")
        if not res_init and glue_opt:  # (glue optimisation works on residue tokens' exit frames)
            raise NotImplementedError("glue optimisation with bond-level init (res_init=False) is not built")
        if not std_bonds and bin_strategy == "uniform":
            raise NotImplementedError("free bonds with uniform (equal-count) bins are not built")
        if glue_opt and glue_opt_method not in ("all", "each"):
            raise ValueError(f"glue_opt_method must be 'all' or 'each', not {glue_opt_method!r}")
        if compute_sec_structs:
            raise NotImplementedError("secondary-structure priorities are not built")
        if isinstance(structures, dict) and "row_off" in structures:
            corpus = structures
            fnames = list(structures["fnames"]) if structures.get("fnames") is not None else None
        else:
            structures = list(structures)
            corpus = structures_to_corpus(structures)
            fnames = [s.get("fname") if isinstance(s, dict) else None for s in structures]
        self._corpus = corpus
        self._fnames = fnames
        self.bins = bins
        self.B = int(bins[1])
        self.bin_strategy = bin_strategy
        self.save_dir = save_dir
        self.compute_sec_structs = compute_sec_structs
        self.plot_iou_with_sec_structs = plot_iou_with_sec_structs
        self.res_init = res_init
        self.std_bonds = std_bonds
        self.rmsd_partition_min_size = rmsd_partition_min_size
        self.rmsd_super_res = bool(rmsd_super_res)
        self.rmsd_only = rmsd_only
        self.num_partitions = ThresholdDict(num_partitions) if isinstance(num_partitions, dict) else num_partitions
        self.max_num_strucs = max_num_strucs
        self.glue_opt = glue_opt
        self.glue_opt_prior = glue_opt_prior
        self.glue_opt_every = glue_opt_every
        self.glue_opt_method = glue_opt_method
        self.seed = seed
        if device is None:  # (with a process group: this rank's own GPU, torchrun's LOCAL_RANK)
            device = int(os.environ.get("LOCAL_RANK", 0)) if group is not None else 0
        self.device = int(device)
        self._group = _RmsdGroup(group, self.device) if group is not None else None
        self.rng = np.random.default_rng(self._group.shared_seed() if self._group is not None and seed is None
                                         else seed)
        self.n = len(corpus["row_off"]) - 1
        self._step = 0
        self._times = []
        self._ious = []
        self._tokens = {}
        self._chains = []
        self._merge_log = []  # [key, count] of every merge popped, recurring repeats included
        self.assign_calls = 0  # device assignment batches (tests check the GPU path ran)

    # ------------------------------------------------------------ geometry on the device
    def _span_coords(self, spans, orig):
        """Tokenizer.compute_coords(index, length, orig) for [(chain, index, length)], one
        device NeRF batch: the span rounded out to whole residues, then its atoms."""
        if isinstance(spans, np.ndarray):  # (_occ_spans' int64 rows)
            return self._span_coords_idx(spans, orig) if len(spans) else []
        if _KEYC is not None and spans and not isinstance(spans[0][0], _Chain):
            return self._span_coords_idx(spans, orig)
        packs, geos, cuts = [], [], []
        for ci, index, length in spans:
            c = ci if isinstance(ci, _Chain) else self._chains[ci]
            length = min(length, 3 * c.n - 1 - index)
            start = 3 * (index // 3)
            end = 3 * (((index + length - 1) + 1) // 3) + 1
            if _KEYC is not None:
                packs.append(self._pack_item((ci, start // 3, (end - start + 2) // 3), orig) if isinstance(ci, int)
                             else (tuple((c.orig if orig else c.cur)[k] for k in _PACK_ORDER), c.init, start // 3,
                                   (end - start + 2) // 3))
            else:
                geos.append(c.geo(start, end - start + 1, orig))
            cuts.append((index - start, end - (index + length - 1)))
        if not cuts:
            return []
        if _KEYC is not None:
            off = np.zeros(len(packs) + 1, dtype=np.int64)
            np.cumsum([p[-1] for p in packs], out=off[1:])
            packed = np.zeros((int(off[-1]), 9), dtype=np.float64)
            _KEYC.pack(packs, packed)
            xyz = _rmsd.nerf_packed(off, packed, device=self.device)
        else:
            xyz = _rmsd.geo_coords(geos, device=self.device)
        return [x[a:len(x) - b] for x, (a, b) in zip(xyz, cuts)]

    def _span_coords_idx(self, spans, orig):
        """_span_coords of spans on chains given by index, in arrays: the NeRF layout packed in
        C (csrc/rmsdkey.c packc), the atoms cut out of the batch's output with one gather.  Spans
        of one atom count (a merge's occurrences) come back as one (n, atoms, 3) array."""
        sp = spans if isinstance(spans, np.ndarray) else np.asarray(spans, dtype=np.int64).reshape(len(spans), 3)
        ci, index = sp[:, 0], sp[:, 1]
        na = self.__dict__.get("_nres_a")
        if na is None or len(na) != len(self._chains):
            na = self._nres_a = np.array([c.n for c in self._chains], dtype=np.int64)
        length = np.minimum(sp[:, 2], 3 * na[ci] - 1 - index)
        start = 3 * (index // 3)
        end = 3 * ((index + length) // 3) + 1
        r = (end - start + 2) // 3
        off = np.zeros(len(sp) + 1, dtype=np.int64)
        np.cumsum(r, out=off[1:])
        packed = np.zeros((int(off[-1]), 9), dtype=np.float64)
        _KEYC.packa(self._chains, bool(orig), np.ascontiguousarray(np.stack([ci, start // 3, r], axis=1)), packed)
        atoms = _rmsd.nerf_atoms(off, packed, device=self.device)
        first = 3 * off[:-1] + (index - start)
        cnt = length + 1
        if (cnt == cnt[0]).all():  # (one flat take: a row gather of 3-double rows is ~3x slower)
            c = int(cnt[0])
            flat = np.ascontiguousarray(atoms).reshape(-1)
            return flat.take((3 * first)[:, None] + np.arange(3 * c)).reshape(len(first), c, 3)
        return [atoms[f:f + c] for f, c in zip(first.tolist(), cnt.tolist())]

    def _occ_spans(self, occ, length):
        """[(ci, token_pos[i2 - 1], length) for (ci, i2) in occ] (bpe.py:1759-1763), as int64
        rows built in C when the extension is there"""
        if _KEYC is not None:
            sp = np.empty((len(occ), 3), dtype=np.int64)
            _KEYC.spans_occ(self._chains, occ, length, sp)
            return sp
        return [(ci, self._chains[ci].token_pos[index - 1], length) for ci, index in occ]

    def _pack_item(self, p, orig):
        ci, q, r = p
        c = self._chains[ci]
        src = c.orig if orig else c.cur
        return (tuple(src[k] for k in _PACK_ORDER), c.init, q, r)

    def _struc_coords(self, strucs):
        """Tokenizer.key_coords(struc) (tokenizer.py:204-230) for medoid geometries that
        start at a residue's N:CA bond: NeRF of the struc, padded to whole residues (the
        padding only places atoms after the kept ones), first num_bonds + 1 atoms."""
        geos, keep = [], []
        for s in strucs:
            nb = sum(len(s.get(k, [])) for k in BOND_TYPES)
            if len(s.get("N:CA", [])) < len(s.get("CA:C", [])) or len(s.get("N:CA", [])) == 0:
                raise NotImplementedError("medoid geometry that does not start at an N:CA bond")
            r = nb // 3 + 1  # whole residues that place atom nb
            g = {k: list(s.get(k, [])) for k in BOND_TYPES + BOND_ANGLES + DIHEDRALS}
            g["N:CA"] += [1.46] * (r - len(g["N:CA"]))
            g["CA:C"] += [1.54] * (r - len(g["CA:C"]))
            g["tau"] += [1.94] * (r - len(g["tau"]))
            for k, v in (("0C:1N", 1.34), ("CA:C:1N", 2.03), ("C:1N:1CA", 2.12), ("psi", 0.0), ("omega", np.pi),
                         ("phi", -1.0)):
                g[k] += [v] * (r - 1 - len(g[k]))
            geos.append(g)
            keep.append(nb + 1)
        xyz = _rmsd.geo_coords(geos, device=self.device)
        return [x[:k] for x, k in zip(xyz, keep)]

    def _assign(self, coords, medoid_coords):
        """_compute_assignment_inner for every occurrence (bpe.py:654-657): argmin over the
        medoids of compute_rmsd(occurrence, medoid) -- one device launch.  With a process
        group each rank takes a contiguous 1/world of the occurrences on its own GPU and the
        assignments are all-gathered (the reference fans this out over a process pool,
        bpe.py:1766-1777); every rank then holds all of them."""
        self.assign_calls += 1
        if len(coords) == 0:
            return []
        g = self._group
        if g is None or g.world == 1:
            return [int(a) for a in _rmsd.assign(coords, medoid_coords, device=self.device)]
        n = len(coords)
        lo, hi = n * g.rank // g.world, n * (g.rank + 1) // g.world
        mine = _rmsd.assign(coords[lo:hi], medoid_coords, device=self.device) if hi > lo else []
        return [int(a) for a in g.gather_chunks(np.asarray(mine, dtype=np.int64), n)]

    # ------------------------------------------------------------ initialize (bpe.py:91-103)
    def initialize(self, path=None):
        from .bpe import BOND_LENGTHS, ThresholdDict
        thr = ThresholdDict()
        for size, grid in self._grid_thresholds().items():
            thr[size] = grid
        if self.std_bonds:  # bpe.py:874-876
            for i, bt in enumerate(BOND_TYPES):
                thr[bt] = [(BOND_LENGTHS[i], BOND_LENGTHS[i])]
        else:  # free bonds: bond-length histograms per grid too (bpe.py:830-831)
            for size, grid in self._bond_thresholds().items():
                thr[size].update(grid)
        self._thresholds = thr
        self._thr_by_len = {}
        self._key_edges = {}
        ro = self._corpus["row_off"]
        init = _rmsd.init_geometry()
        self._chains = []
        for r in range(self.n):
            cols = {c: np.asarray(self._corpus[c][ro[r]:ro[r + 1]], dtype=np.float64) for c in COLUMNS}
            self._chains.append(_Chain(cols, init, self._fnames[r] if self._fnames else None))
        if self.res_init:
            self._init_residues()
        else:
            self._init_bonds()
        return self

    def _init_bonds(self):
        """_init_tokens (bpe.py:397-420), res_init=False: every bond its own initial token --
        token ids 0, 1, 2 = {N:CA: [0]}, {CA:C: [0]}, {0C:1N: [0]} by the bond's type
        (Tokenizer.bond_labels, tokenizer.py:49) -- each bond set to its type's standard length
        (std_bonds); the angles stay raw (the glue snap is the residue init's, bpe.py:381-391)."""
        self._tokens = {i: {BOND_TYPES[i]: [0]} for i in range(3)}
        std = {bt: sum(self._thresholds[bt][0]) / 2 for bt in BOND_TYPES}
        for c in self._chains:
            c.init[0], c.init[1] = std["N:CA"], std["CA:C"]
            for bt in BOND_TYPES:
                c.cur[bt][:max(c.n - 1, 0)] = [std[bt]] * max(c.n - 1, 0)
            c.btt = {j: (j, j % 3, 1) for j in range(3 * c.n - 1)}
            c.token_pos = list(range(3 * c.n - 1))
            c.tokens0 = list(c.btt.values())

    def _grid_thresholds(self):
        """{size: thresholds} of the six angle types for every grid of ``bins``
        (bpe.py:820-876): the device min / max / count pass of the scoped mode's engine,
        then np.histogram edges with each size's bin count on the host."""
        from .engine import GeoBPEEngine
        e = GeoBPEEngine(self._corpus, self.B, device=self.device, strategy=self.bin_strategy)
        try:
            e.initialize()
            return {s: ({k: list(v) for k, v in e.thresholds.items()} if s == 1 else e.thresholds_for(b))
                    for s, b in self.bins.items()}
        finally:
            e.close()

    def _bond_thresholds(self):
        """{size: {bond type: thresholds}} with free bonds: np.histogram edges of every
        chain's bond lengths (zeros / NaN padding dropped, the chain's two init lengths
        added; bpe.py:841-852, plotting.py:316-319 non-circular) per grid's bin count.  An
        order statistic of the host copy of the input, like the uniform strategy's edges."""
        ro = self._corpus["row_off"]
        n_ca, ca_c, _ = _rmsd.init_geometry()
        out = {s: {} for s in self.bins}
        for bt in BOND_TYPES:
            col = np.asarray(self._corpus[bt], dtype=np.float64)
            vals = col[np.nan_to_num(col, nan=0.0) != 0.0]
            if bt in ("N:CA", "CA:C"):
                vals = np.concatenate([vals, np.full(len(ro) - 1, n_ca if bt == "N:CA" else ca_c)])
            for s, b in self.bins.items():
                e = np.histogram_bin_edges(vals, bins=int(b))
                out[s][bt] = [(float(a), float(c)) for a, c in zip(e[:-1], e[1:])]
        return out

    def _centre(self, k, ind, size):
        lookup = self._thresholds if k in BOND_TYPES and self.std_bonds else self._thresholds[size]
        return sum(lookup[k][ind]) / 2

    def _init_residues(self):
        p = self.rmsd_partition_min_size
        for c in self._chains:  # every bond -> its bin centre (bpe.py:714-737)
            if self.std_bonds:  # bonds 0, 1 (the init lengths) and rows 0..n-2 of the three columns
                std = {bt: sum(self._thresholds[bt][0]) / 2 for bt in BOND_TYPES}
                c.init[0], c.init[1] = std["N:CA"], std["CA:C"]
                for bt in BOND_TYPES:
                    c.cur[bt][:max(c.n - 1, 0)] = [std[bt]] * max(c.n - 1, 0)
                continue
            for j in range(3 * c.n - 1):  # free bonds: grid 1's bin of the length (strict get_ind, bpe.py:731)
                bt = BOND_TYPES[j % 3]
                v = self._centre(bt, _get_ind(c.geo(j, 1)[bt][0], self._thresholds[1][bt]), 1)
                c.set_geo(j, 1, {bt: [v]})
        if self.glue_opt and self.glue_opt_method == "all":  # exit frames, bond-standardized (bpe.py:192-229)
            from .glue import exit_frames
            self._exit_frames = exit_frames(self._chains, device=self.device)
        label_dict, res_geo, labels = {}, {}, []
        for ci, c in enumerate(self._chains):
            lab = []
            for i in range(c.n):
                start, length = 3 * i, (3 if i < c.n - 1 else 2)
                if length < p:  # binned residue (bpe.py:237-249)
                    if not self.std_bonds:  # quant_geo reads _thresholds[bond] (bpe.py:1518-1524)
                        raise KeyError("N:CA")
                    geo = c.geo(start, length)
                    cen = {}
                    for k, vals in geo.items():
                        q = []
                        for v in vals:
                            if k in BOND_TYPES:
                                q.append(_get_ind(v, self._thresholds[k]))
                            else:
                                q.append(_get_ind((v + TWO_PI) % TWO_PI, self._thresholds[length][k]))
                        cen[k] = [self._centre(k, x, length) for x in q]
                    s = json.dumps(cen, sort_keys=True)
                    n = label_dict.setdefault(s, len(label_dict))
                    c.set_geo(start, length, cen)
                    lab.append(n)
                else:
                    res_geo.setdefault(length, []).append((ci, start, length))
                    lab.append(None)
            labels.append(lab)
        for ci, c in enumerate(self._chains):
            c.btt = {3 * i: (3 * i, labels[ci][i], 3 if i < c.n - 1 else 2) for i in range(c.n)}
            c.token_pos = [3 * (j // 3) for j in range(3 * c.n - 1)]
        if res_geo and self.glue_opt and self.glue_opt_method == "each" and \
                any(start > 0 for occ in res_geo.values() for _, start, _ in occ):
            # the reference's "each" method calls opt_glue without bin centres in the main
            # process (bpe.py:365-369) and stops at its assert (bpe.py:761); with p >= 4 no
            # residue is partitioned and the first RMSD merge raises AttributeError instead
            raise AssertionError("opt_glue: bin_centers is None and BIN_CENTERS is not set (bpe.py:761)")
        if res_geo:
            self._sphere_dict = {}
            self._tokens = {}
            for n, size in enumerate(res_geo):
                self._partition_residues(n, size, res_geo[size])
        for c in self._chains:
            c.tokens0 = list(c.btt.values())
        for c in (self._chains if not (res_geo and self.glue_opt) else []):
            # glue angles -> grid-1 bin centres, NaN kept (bpe.py:381-391); with glue_opt and
            # partitioned residues they stay raw until glue_opt_all snaps them
            for k in GLUE:
                col = c.cur[k]
                for r in range(c.n):
                    v = col[r]
                    if v == v:
                        col[r] = self._centre(k, _get_ind((v + TWO_PI) % TWO_PI, self._thresholds[1][k]), 1)
        if not res_geo:
            self._tokens = {n: json.loads(s) for s, n in label_dict.items()}

    # ------------------------------------------------------------ glue optimisation
    def glue_opt_all(self):
        """BPE.glue_opt_all (bpe.py:106-135): every chain's glues optimised against its
        cached exit frames (bin/encode.py:331-332 calls it after initialize())."""
        self._glue_opt(range(self.n))

    def _glue_prior_tables(self):
        """_bin_centers / _bin_weights of every grid (bpe.py:834-872) as device tables."""
        if not hasattr(self, "_glue_prior"):
            from . import glue as G
            sizes = sorted(self.bins)
            counts = self._bin_count_values()
            self._glue_prior = G.prior_tables([self._thresholds[s0] for s0 in sizes], [counts[s0] for s0 in sizes])
        return self._glue_prior

    def _glue_opt(self, cis, chains=None, frames=None):
        """_opt_glue_worker + opt_glue (bpe.py:739-807) for the chains cis (or the given
        chain objects and their cached frames), as one device launch: glue k = (omega_k,
        C:1N:1CA_k, phi_{k+1}) of every initial token but the last, started from the current
        values, aimed at exit frame (start + length) // 3 - 1 of the cached chain; the optimum
        snapped to grid(3n - 4)'s bins and written back.  Returns cis."""
        from . import glue as G
        cis = list(cis)
        if chains is None:
            chains = [self._chains[ci] for ci in cis]
            frames = [self._exit_frames[ci] for ci in cis]
        if not chains:
            return cis
        sizes = sorted(self.bins)
        geos, x0s, tgts, grids = [], [], [], []
        for c, (R, t) in zip(chains, frames):
            g = G.pack_chain(c.cur, c.init)
            toks = c.tokens0[:-1]
            geos.append(g)
            x0s.append(np.stack([[c.cur["omega"][(i + ln) // 3 - 1], c.cur["C:1N:1CA"][(i + ln) // 3 - 1],
                                  c.cur["phi"][(i + ln) // 3]] for i, _, ln in toks]).astype(np.float32)
                       if toks else np.zeros((0, 3), np.float32))
            rows = [(i + ln) // 3 - 1 for i, _, ln in toks]  # R_occs[res_no - 2], bpe.py:751-755
            tgts.append((R[rows], t[rows]))
            L = 3 * c.n - 4
            grids.append(max([k for k in sizes if k <= L], default=sizes[0]))
        if any(len(x) != len(g) - 1 for x, g in zip(x0s, geos)):
            raise NotImplementedError("glue opt over initial tokens other than one per residue")
        lam = float(self.glue_opt_prior) if self.glue_opt_prior and self.glue_opt_prior > 0.0 else 0.0
        outs, _, _ = G.optimize_chains(geos, x0s, tgts, [sizes.index(k) for k in grids], self._glue_prior_tables(),
                                       lam, device=self.device)
        self.glue_calls = getattr(self, "glue_calls", 0) + 1
        for c, opt, gk in zip(chains, outs, grids):
            thr = self._thresholds[gk]
            om, cn, ph = (G.snap_many(thr[k], opt[:, t]).tolist() for t, k in enumerate(G.GLUE))
            for k, (i, _, ln) in enumerate(c.tokens0[:-1]):
                row = (i + ln) // 3 - 1
                c.cur["omega"][row] = om[k]
                c.cur["C:1N:1CA"][row] = cn[k]
                c.cur["phi"][row + 1] = ph[k]
        return cis

    def _partition_residues(self, n, size, occ):
        """The res_geo partition of one residue size (bpe.py:266-379)."""
        if size not in RES_SPHERE_KEY:
            raise NotImplementedError(f"residue size {size}")
        N = len(occ)
        active = (self.rng.choice(N, self.max_num_strucs, replace=False) if N > self.max_num_strucs
                  else np.arange(N))
        sup = self.rmsd_super_res
        coords = self._span_coords(occ, sup)
        act = coords[active] if isinstance(coords, np.ndarray) else [coords[i] for i in active]
        k = self.num_partitions[size]
        medoids = _rmsd.k_medoids(act, k, rng=self.rng, device=self.device)
        if len(medoids) not in (1, k):
            # the reference stores the medoids in a memmap of num_partitions[size] entries
            # (bpe.py:299-300): numpy broadcasts one medoid into it (one structure of the
            # size: the run goes on with that medoid list), any other shortfall fails the write
            raise ValueError(f"could not broadcast input array from shape ({len(medoids)},) into shape ({k},)")
        assign = self._assign(coords, [act[m] for m in medoids])
        key = RES_SPHERE_KEY[size]
        self._sphere_dict[key] = []
        for p, m in enumerate(medoids):
            ci, start, length = occ[int(active[m])]
            struc = self._chains[ci].geo(start, length, sup)
            self._sphere_dict[key].append(struc)
            self._tokens[(n, p)] = struc
        for (ci, start, length), p in zip(occ, assign):
            c = self._chains[ci]
            c.set_geo(start, length, self._tokens[(n, p)])
            c.btt[start] = (start, (n, p), length)

    # ------------------------------------------------------------ keys (bpe.py:1192-1299)
    def _pair_key(self, ci, idx1, l1, l2):
        c = ci if isinstance(ci, _Chain) else self._chains[ci]
        idx2 = idx1 + l1
        t1, t2 = c.btt[c.token_pos[idx1]], c.btt[c.token_pos[idx2]]
        if t1[0] == t2[0]:
            raise RuntimeError("pair of one token")  # the reference stops in breakpoint() here
        pt1, pt2 = isinstance(t1[1], tuple), isinstance(t2[1], tuple)
        L = l1 + l2
        # which span items are quantized (bpe.py:1247-1285), as a range [lo, hi) of the
        # item's index i within the span, per kind (bond, angle, dihedral)
        if pt1 and pt2:
            rng = ((0, 0), (l1 - 1, l1), (l1 - 2, l1))
        elif pt1:
            rng = ((l1, L), (l1 - 1, L), (l1 - 2, L))
        elif pt2:
            rng = ((0, l1), (0, l1), (0, l1))
        else:
            rng = ((0, L), (0, L), (0, L))
        if _KEYC is not None and not self._py_keys:
            if idx1 + L - 1 > 3 * c.n - 1:
                raise ValueError(f"idx+l cannot exceed {3 * c.n - 1}")
            edges = self._key_edges.get(L)
            if edges is None:
                edges = self._key_edges[L] = self._edges_for(L)
            cur = c.cur
            return _KEYC.key(tuple(cur[k] for k in _KEY_ORDER), c.init, idx1, L, idx1 % 3, rng, edges)
        return self._pair_key_py(c, idx1, L, rng)

    def _edges_for(self, L):
        """The (left edges, right edges) lists of every item type's thresholds at span length L,
        in json key order (rmsdkey.c's layout).  For a type whose thresholds do not exist the
        entry is the exception the lookup raised: rmsdkey.c raises it when such a type is
        binned, so the C key and the C merge loop fail as _pair_key_py (the reference) does."""
        thr_all = self._thresholds
        thr_L = self._thr_by_len.get(L)
        if thr_L is None:
            thr_L = self._thr_by_len[L] = thr_all[L]
        out = []
        for k in _KEY_ORDER:
            kind = _ITEM[k][1]
            try:
                thr = (thr_all[k] if self.std_bonds else thr_L[k]) if kind == 0 else thr_L[k]
                out.append(([float(a) for a, _ in thr], [float(b) for _, b in thr]))
            except (KeyError, TypeError) as e:
                out.append(e.with_traceback(None))
        return tuple(out)

    def _edges_store(self, L):
        """_edges_for(L), cached (called by csrc/rmsdkey.c merge for a length it has not seen)."""
        e = self._key_edges[L] = self._edges_for(L)
        return e

    def _pair_key_py(self, c, idx1, L, rng):
        """_pair_key in Python: the restatement rmsdkey.c follows (and the path taken for
        its errors, so the reference's exceptions surface unchanged)."""
        geo = c.geo(idx1, L)
        ph = idx1 % 3
        thr_all = self._thresholds
        thr_L = self._thr_by_len.get(L)
        if thr_L is None:
            thr_L = self._thr_by_len[L] = thr_all[L]
        for k, vals in geo.items():
            t0, kind = _ITEM[k]
            lo, hi = rng[kind]
            if lo >= hi:
                continue
            base = (t0 + 3 - ph) % 3
            m_lo = max(0, -((base - lo) // 3))      # first m with base + 3m >= lo
            m_hi = min(len(vals), -((base - hi) // 3))
            if m_lo >= m_hi:
                continue
            thr = (thr_all[k] if self.std_bonds else thr_L[k]) if kind == 0 else thr_L[k]
            out = list(vals)
            for m in range(m_lo, m_hi):
                v = vals[m]
                out[m] = _get_ind(v, thr) if kind == 0 else _get_ind((v + TWO_PI) % TWO_PI, thr)
            geo[k] = out
        return _ENC.encode(geo)

    # ------------------------------------------------------------ bin (bpe.py:1431-1474)
    def bin(self):
        self._geo_dict = defaultdict(set)
        # the key of every live pair by (chain, start of its second token): a pair's key
        # changes only when a merge replaces the pair, so step() reads the old neighbour keys
        # from here instead of re-deriving them from the geometry (bpe.py:1917, 1933, 1941).
        # One list per chain indexed by bond (None: no pair starts there) -- a merge's
        # occurrences read and write their chain's list instead of hashing (chain, bond)
        # tuples into one dict of every pair
        self._pk = [[None] * (3 * c.n) for c in self._chains]
        for ci, c in enumerate(self._chains):
            toks = c.tokens()
            for (i1, _, l1), (i2, _, l2) in zip(toks, toks[1:]):
                k = self._pair_key(ci, i1, l1, l2)
                self._geo_dict[k].add((ci, i2))
                self._pk[ci][i2] = k
        self._geo_step = {k: 0 for k in self._geo_dict}
        self._key_to_priority = {key: (True, -len(occ), key) for key, occ in self._geo_dict.items()}
        self._priority = _PrioQueue(self._key_to_priority)
        self._sphere_keys = {}

    @property
    def _priority_dict(self):
        """The reference's SortedDict of priorities, as its sorted key view."""
        return list(self._priority)

    # ------------------------------------------------------------ step (bpe.py:1792-2166)
    def step(self):
        # (the cyclic collector is paused for the step: a step allocates thousands of tracked
        # tuples, and the full passes they set off over the tracked host state -- millions of
        # pair tuples, sets and dicts -- were a quarter of a 2000-chain step; nothing here makes
        # cycles, refcounting frees it all, and the collector resumes as it was)
        gc_was = gc.isenabled()
        gc.disable()
        try:
            while True:
                self._merge()
                if not len(self._priority):
                    raise IndexError("peekitem on an empty priority dict (bpe.py:2164)")
                if self._priority[0][0]:
                    return
        finally:
            if gc_was:
                gc.enable()

    def _partition(self, key, length):
        """rmsd_partition (bpe.py:1739-1789): k-medoids over (a sample of) the occurrences,
        every occurrence assigned to its nearest medoid, the medoids' geometry recorded."""
        occ = list(self._geo_dict[key])
        N = len(occ)
        active = (self.rng.choice(N, self.max_num_strucs, replace=False) if N > self.max_num_strucs
                  else np.arange(N))
        spans = self._occ_spans(occ, length)
        sup = self.rmsd_super_res
        coords = self._span_coords(spans, sup)
        act = coords[active] if isinstance(coords, np.ndarray) else [coords[i] for i in active]
        medoids = _rmsd.k_medoids(act, self.num_partitions[length], rng=self.rng, device=self.device)
        assign = self._assign(coords, [act[m] for m in medoids])
        strucs = []
        for m in medoids:
            ci, i1 = (int(x) for x in spans[int(active[m])][:2])
            strucs.append(self._chains[ci].geo(i1, length, sup))
        self._sphere_dict[key] = strucs
        return occ, assign

    def _merge(self):
        t0 = time.time()
        if not len(self._priority):
            raise IndexError("peekitem on an empty priority dict")
        flag, negc, key = self._priority[0]
        recurring = not flag
        self._merge_log.append([key, -negc])
        key_dict = json.loads(key)
        length = sum(len(key_dict.get(k, [])) for k in BOND_TYPES)
        rmsd = length >= self.rmsd_partition_min_size
        if rmsd:
            if not hasattr(self, "_sphere_dict"):
                # p >= 4: the reference never creates _sphere_dict (bpe.py:264, 1780)
                raise AttributeError("'BPE' object has no attribute '_sphere_dict'")
            if recurring:
                occ = list(self._geo_dict[key])
                spans = self._occ_spans(occ, length)
                assign = self._assign(self._span_coords(spans, self.rmsd_super_res),
                                      self._struc_coords(self._sphere_dict[key]))
            else:
                occ, assign = self._partition(key, length)
        n = len(self._tokens)
        if not rmsd:
            binned = {k: [self._centre(k, v, length) if isinstance(v, int) else v for v in vals]
                      for k, vals in key_dict.items()}
            self._tokens[n] = key_dict
        elif recurring:
            n = sorted({k[0] for k in self._tokens})[list(self._sphere_dict).index(key)]
        else:
            for p, struc in enumerate(self._sphere_dict[key]):
                self._tokens[(n, p)] = struc
        if not rmsd:
            occ = list(self._geo_dict[key])
        diff = {}

        def note(k, d):
            diff[k] = diff.get(k, 0) + d

        gd = self._geo_dict
        # without RMSD partitioning, a multi-grid schedule re-snaps a merged span after its
        # neighbour keys were computed (bpe.py:2010-2013), so stored keys can go stale: then
        # every key is derived afresh from the geometry, as the reference does
        stale_ok = not rmsd and len(self.bins) > 1
        last_ci = last_i1 = None
        order = sorted(range(len(occ)), key=occ.__getitem__)
        if _KEYC is not None and not stale_ok and not self._py_keys:
            # the loop below in C (csrc/rmsdkey.c merge), on these same sets / dicts / lists
            # (the pair-key memo of rmsdkey.c: partitioned tokens keep their medoid geometry
            # unless glue optimisation rewrites the glues inside them)
            memo = None
            if not self.glue_opt and not self.rmsd_only and not self._no_key_memo:
                memo = self.__dict__.get("_key_memo")
                if memo is None:
                    memo = self._key_memo = _KEYC.memo_new()
            _KEYC.merge((self._chains, gd, self._pk, self._key_edges, self._edges_store, _KEY_ORDER_T, memo),
                        [occ[i] for i in order], [assign[i] for i in order] if rmsd else None, key, length, n,
                        rmsd, (None if self.rmsd_only else self._sphere_dict[key]) if rmsd else binned, diff)
            order = ()
        for idx in order:
            ci, i2 = occ[idx]
            c = self._chains[ci]
            tp = c.token_pos
            i1 = tp[i2 - 1]
            l1 = i2 - i1
            l2 = length - l1
            overlaps = last_ci == ci and last_i1 + length > i1
            # (overlaps != not present: the reference calls breakpoint() and, with breakpoints
            # off, carries on, bpe.py:1909-1912; only stale multi-grid keys get here)
            if overlaps:
                continue
            if not (l1 > 0 and l2 > 0):
                raise AssertionError("bad split")
            pk = self._pk[ci]
            if pk[i2] != key or (stale_ok and self._pair_key(ci, i1, l1, l2) != key):
                # bpe.py:1917-1920 (breakpoint(); continue): the stored key is the pair's key
                # unless a multi-grid re-snap made it stale (no RMSD partitioning)
                continue
            gd[key].remove((ci, i2))
            pk[i2] = None
            note(key, -1)
            left = right = None
            if i1:
                i0 = tp[i1 - 1]
                l0 = i1 - i0
                left = self._pair_key(ci, i0, l0, l1) if stale_ok else _pk_at(pk, ci, i1)
            if i2 + l2 < len(tp):
                i3 = i2 + l2
                l3 = 0
                while i3 + l3 < len(tp) and tp[i3 + l3] == i3:
                    l3 += 1
                right = self._pair_key(ci, i2, l2, l3) if stale_ok else _pk_at(pk, ci, i3)
            if left:
                gd[left].remove((ci, i1))
                note(left, -1)
            if right:
                gd[right].remove((ci, i3))
                note(right, -1)
            for j in range(i2, i2 + l2):
                tp[j] = i1
            c.btt.pop(i2)
            c.btt[i1] = (i1, (n, assign[idx]) if rmsd else n, length)
            c.events.append((i1, i2, c.btt[i1]))
            if rmsd and not self.rmsd_only:  # (bpe.py:1977)
                c.set_geo(i1, length, self._sphere_dict[key][assign[idx]])
            if left:
                k = self._pair_key(ci, i0, l0, length)
                gd[k].add((ci, i1))
                pk[i1] = k
                note(k, +1)
            if right:
                k = self._pair_key(ci, i1, length, l3)
                gd[k].add((ci, i3))
                pk[i3] = k
                note(k, +1)
            if not rmsd:
                c.set_geo(i1, length, binned)
            last_ci, last_i1 = ci, i1
        # glue re-optimisation of every chain the merge touched (bpe.py:2027-2071): all glues
        # of each chain, then every adjacent token pair whose key changed moves between sets
        if (rmsd and self.glue_opt and not self.rmsd_only and self.glue_opt_method == "all"
                and self._step % self.glue_opt_every == 0):
            uniq = set(ci for ci, _ in occ)
            cis = self._glue_opt(list(uniq))
            if _KEYC is not None and not self._py_keys:  # (the loop below in C: csrc/rmsdkey.c rekey)
                _KEYC.rekey((self._chains, gd, self._pk, self._key_edges, self._edges_store, _KEY_ORDER_T, None),
                            list(cis), diff)
                cis = ()
            for ci in cis:
                btt = self._chains[ci].btt
                pk = self._pk[ci]
                last = 3 * self._chains[ci].n - 1
                for i1, (_, _, l1) in list(btt.items()):
                    if i1 + l1 == last:
                        continue
                    i2 = i1 + l1
                    l2 = btt[i2][2]
                    old = _pk_at(pk, ci, i2)
                    new = self._pair_key(ci, i1, l1, l2)
                    if new != old:
                        gd[old].remove((ci, i2))
                        note(old, -1)
                        gd[new].add((ci, i2))
                        pk[i2] = new
                        note(new, +1)
        if not recurring:
            self._step += 1
        if _KEYC is not None and not self._py_keys:  # (step 7 below, in C on the same objects)
            _KEYC.prio(diff, self._key_to_priority, self._priority.heap, heapq.heappush, gd,
                       getattr(self, "_sphere_dict", {}))
            diff = {}
        for k, d in diff.items():  # step 7 (bpe.py:2077-2138)
            pr = self._key_to_priority.pop(k, None)
            count = 0
            if pr is not None:
                self._priority.remove(pr)
                count = -pr[1]
            count += d
            if count != len(gd[k]):
                raise AssertionError(f"count of {k[:60]} out of step")
            if count:
                pr = (k not in getattr(self, "_sphere_dict", {}), -count, k)
                self._key_to_priority[k] = pr
                self._priority.add(pr)
            else:
                gd.pop(k)
        self._times.append(time.time() - t0)

    def run(self, n_steps: int) -> int:
        """n step() calls (bin/encode.py's loop, bpe.py:398); stops early when no pair is
        left.  Returns the calls completed."""
        done = 0
        for _ in range(n_steps):
            if not len(self._priority):
                break
            try:
                self.step()
            except IndexError:  # the last merge emptied the priority dict (bpe.py:2164)
                done += 1
                break
            done += 1
        return done

    @property
    def merges(self):
        """[(key string, count)] of every merge, recurring repeats included."""
        return [tuple(m) for m in self._merge_log]

    # ------------------------------------------------------------ induce (bpe.py:1053-1140)
    def tokenize(self, structure):
        """BPE.tokenize: a new chain segmented with the trained vocabulary.  Its bonds go
        to their bins (out-of-range lengths clamp, ``strict=False``); every residue is
        assigned to its nearest residue medoid (device NeRF + RMSD); the glue angles go to
        grid-1 centres; then every merge key, in training order, is applied to the chain
        alone (``step_helper``, bpe.py:1316-1425: nearest medoid per occurrence, greedy left
        to right, the medoid's geometry written back).  Returns (tokenizer, metrics) with
        metrics["L"] = the token count before and after each key; the reference's backbone
        RMSD / lDDT against the PDB need esm's ProteinChain and are not computed.

        ``structure``: {"angles": 9 columns, "fname": ...} (the reference's structure
        dict) or a mapping of the 9 columns."""
        if not self.res_init:
            raise NotImplementedError
        ang = structure["angles"] if isinstance(structure, dict) and "angles" in structure else structure
        fname = structure.get("fname") if isinstance(structure, dict) else None
        c = _Chain({k: np.asarray(ang[k], dtype=np.float64) for k in COLUMNS}, _rmsd.init_geometry(), fname)
        for j in range(3 * c.n - 1):  # _set_bond_length_worker(t, strict=False) (bpe.py:715-737)
            bt = BOND_TYPES[j % 3]
            if self.std_bonds:
                v = sum(self._thresholds[bt][0]) / 2
            else:
                thr = self._thresholds[1][bt]
                x = c.geo(j, 1)[bt][0]
                ind = 0 if x < thr[0][0] else (len(thr) - 1 if x > thr[-1][1] else _get_ind(x, thr))
                v = sum(thr[ind]) / 2
            c.set_geo(j, 1, {bt: [v]})
        if self.glue_opt and self.glue_opt_method == "each" and c.n > 1:
            # opt_glue without bin centres in this process (bpe.py:1090-1093, 761)
            raise AssertionError("opt_glue: bin_centers is None and BIN_CENTERS is not set (bpe.py:761)")
        frames = None
        if self.glue_opt:  # t.cached_all_frames (bpe.py:1062-1063)
            from .glue import exit_frames
            frames = exit_frames([c], device=self.device)
        res_geo = {}
        for i in range(c.n):
            res_geo.setdefault(3 if i < c.n - 1 else 2, []).append(3 * i)
        c.token_pos = [3 * (j // 3) for j in range(3 * c.n - 1)]
        c.btt = {3 * i: (3 * i, None, 3 if i < c.n - 1 else 2) for i in range(c.n)}
        for n, size in enumerate(res_geo):  # nearest residue medoid (bpe.py:1072-1099)
            geo = c.geo(0, 5) if size == 3 else c.geo(0, 2)
            strucs = []
            p = 0
            while (n, p) in self._tokens:
                key = self._tokens[(n, p)]
                for k in key:
                    geo[k][:len(key[k])] = key[k]
                strucs.append({k: list(v) for k, v in geo.items()})
                p += 1
            med = [x[:size + 1] for x in _rmsd.geo_coords(strucs, device=self.device)]
            starts = res_geo[size]
            assign = self._assign(self._span_coords([(c, s0, size) for s0 in starts], False), med)
            for s0, p in zip(starts, assign):
                c.set_geo(s0, size, self._tokens[(n, p)])
                c.btt[s0] = (s0, (n, p), size)
        c.tokens0 = list(c.btt.values())
        if self.glue_opt:  # glue_opt "all" (bpe.py:1109-1112)
            self._glue_opt([0], [c], frames)
        for k in (GLUE if not self.glue_opt else []):  # grid-1 glue centres, NaN kept (bpe.py:1101-1108)
            col = c.cur[k]
            for r in range(c.n):
                v = col[r]
                if v == v:
                    col[r] = self._centre(k, _get_ind((v + TWO_PI) % TWO_PI, self._thresholds[1][k]), 1)
        geo_dict = defaultdict(set)  # bin_helper (bpe.py:1301-1314)
        toks = c.tokens()
        for (i1, _, l1), (i2, _, l2) in zip(toks, toks[1:]):
            geo_dict[self._pair_key(c, i1, l1, l2)].add(i2)
        uniq = sorted({k[0] for k in self._tokens})
        keys = list(self._sphere_dict)
        if len(uniq) != len(keys):
            raise AssertionError("_tokens and _sphere_dict out of step")
        metrics = {"L": [len(c.btt)]}
        count = 0
        for n, key in zip(uniq[2:], keys[2:]):
            if key in geo_dict:
                self._step_helper(geo_dict, c, key, n, opt=count % self.glue_opt_every == 0, frames=frames)
                count += 1
            metrics["L"].append(len(c.btt))
        return RmsdTokenizer(c, self.device), metrics

    def _step_helper(self, geo_dict, c, key, n, opt=False, frames=None):
        """step() on one chain for a trained key (bpe.py:1316-1425), with the glue
        re-optimisation of glue_opt "all" when opt (bpe.py:1405-1424)."""
        key_dict = json.loads(key)
        length = sum(len(key_dict.get(k, [])) for k in BOND_TYPES)
        vals = list(geo_dict[key])
        tp = c.token_pos
        spans = [(c, tp[index - 1], length) for index in vals]
        assign = self._assign(self._span_coords(spans, self.rmsd_super_res), self._struc_coords(self._sphere_dict[key]))
        last_i1 = None
        for idx in sorted(range(len(vals)), key=vals.__getitem__):
            i2 = vals[idx]
            i1 = tp[i2 - 1]
            l1 = i2 - i1
            l2 = length - l1
            overlaps = last_i1 is not None and last_i1 + length > i1
            if overlaps != (i2 not in geo_dict[key]):
                raise RuntimeError("occurrence bookkeeping out of step (the reference stops in breakpoint())")
            if overlaps:
                continue
            if not (l1 > 0 and l2 > 0):
                raise AssertionError("bad split")
            if self._pair_key(c, i1, l1, l2) != key:
                continue  # bpe.py:1350-1352
            geo_dict[key].remove(i2)
            left = right = None
            if i1:
                i0 = tp[i1 - 1]
                l0 = i1 - i0
                left = self._pair_key(c, i0, l0, l1)
            if i2 + l2 < len(tp):
                i3 = i2 + l2
                l3 = 0
                while i3 + l3 < len(tp) and tp[i3 + l3] == i3:
                    l3 += 1
                right = self._pair_key(c, i2, l2, l3)
            if left:
                geo_dict[left].remove(i1)
            if right:
                geo_dict[right].remove(i3)
            for j in range(i2, i2 + l2):
                tp[j] = i1
            c.btt.pop(i2)
            c.btt[i1] = (i1, (n, assign[idx]), length)
            c.events.append((i1, i2, c.btt[i1]))
            if not self.rmsd_only:  # bpe.py:1386: rmsd_only keeps the occurrence's own geometry
                c.set_geo(i1, length, self._sphere_dict[key][assign[idx]])
            if left:
                geo_dict[self._pair_key(c, i0, l0, length)].add(i1)
            if right:
                geo_dict[self._pair_key(c, i1, length, l3)].add(i3)
            last_i1 = i1
        if self.glue_opt and self.glue_opt_method == "all" and opt and not self.rmsd_only:
            toks = c.tokens()
            old = [self._pair_key(c, i1, l1, l2) for (i1, _, l1), (_, _, l2) in zip(toks, toks[1:])]
            self._glue_opt([0], [c], frames)
            for ((i1, _, l1), (i2, _, l2)), ok in zip(zip(toks, toks[1:]), old):
                nk = self._pair_key(c, i1, l1, l2)
                if nk != ok:
                    geo_dict[ok].remove(i2)
                    geo_dict[nk].add(i2)

    # ------------------------------------------------------------ views / encode
    @property
    def tokenizers(self):
        return [RmsdTokenizer(c, self.device) for c in self._chains]

    init_structure = staticmethod(init_structure)

    def recover_structure(self, repl, tokenized):
        """bpe.py:1029-1051 (bin/train.py:715-716)."""
        return recover_structure(self._tokens, repl, tokenized, self.device)

    @property
    def vocab_size(self):
        return len(self._tokens) + self.cum_bin_count()

    def cum_bin_count(self, key=None):
        from .bpe import BPE
        return BPE.cum_bin_count(self, key)

    def quantize(self, tokenized):
        """bpe.py:928-956 (MOTIF ids by position in _tokens: a token id that is not in
        _tokens -- p = 3 leaves the binned last residues out -- raises ValueError there too)."""
        from .bpe import BPE
        if isinstance(tokenized, RmsdTokenizer):
            return BPE._quantize_tuples(self, tokenized.tokenize())
        if len(tokenized) and isinstance(tokenized[0], RmsdTokenizer):
            return [BPE._quantize_tuples(self, t.tokenize()) for t in tokenized]
        return BPE._quantize_tuples(self, tokenized)

    def dequantize(self, quantized):
        from .bpe import BPE
        return BPE.dequantize(self, quantized)

    def recover(self, tokenized):
        from .bpe import BPE
        return BPE.recover(self, tokenized)

    def encode_all(self):
        """quantize(tokenize()) of every chain as (ids, row offsets)."""
        q = [self.quantize(t) for t in self.tokenizers]
        off = np.zeros(len(q) + 1, dtype=np.int64)
        np.cumsum([len(x) for x in q], out=off[1:])
        return np.array([i for x in q for i in x], dtype=np.int64), off

    def capacity(self, tokenizer=False):
        from .bpe import BPE
        return BPE.capacity(self, tokenizer)

    # ------------------------------------------------------------ checkpoints
    def checkpoint_object(self):
        """The reference's BPE object graph of this run (what bin/encode.py pickles,
        bpe.py:33-88 + the RMSD mode's _sphere_dict): tokenizers with their current and
        original frames, init triple, initial tokens, token_pos and bond_to_token holding the
        merge tree; _tokens, _sphere_dict, _geo_dict, _priority_dict, _key_to_priority,
        _geo_step, the per-grid thresholds / bin counts / centres / weights, and the rng in
        its current state -- so the reference resumes this run (tests/test_rmsd_mode.py)."""
        import pandas as pd
        import torch
        from sortedcontainers import SortedDict

        from . import refpickle as R
        C = R._real_or_local()
        glue = self.glue_opt and self.glue_opt_method == "all"
        toks = [self.tokenizer_record(c, C, self._exit_frames[i] if glue else None, bool(self.glue_opt))
                for i, c in enumerate(self._chains)]
        return self._bpe_record(toks, C)

    @staticmethod
    def tokenizer_record(c, C=None, frames=None, glue_opt=False):
        """The reference Tokenizer object of one chain (tokenizer.py:24-61 attributes, the
        frames, bond_to_token with the merge tree; with glue opt the cached exit frames,
        ``cached_all_frames`` = (R_occs, t_occs), bpe.py:742-748, 1063)."""
        import pandas as pd

        from . import refpickle as R
        if isinstance(c, RmsdTokenizer):
            c = c._c
        C = C or R._real_or_local()
        tok = R._new(C["Tokenizer"], {})
        nodes = {v[0]: R._new(C["Node"], {"value": v, "left": None, "right": None}) for v in c.tokens0}
        leaves = {v[0]: R._new(C["Node"], {"value": v, "left": None, "right": None}) for v in c.tokens0}
        for a, b, v in c.events:  # BinaryTreeBuilder.combine
            left, right = nodes.pop(a), nodes.pop(b)
            nodes[v[0]] = R._new(C["Node"], {"value": v, "left": left, "right": right})
        tree = R._new(C["BinaryTreeBuilder"], {"nodes": nodes, "leaves": leaves})
        hier = R._new_dict(C["TokenHierarchy"], list(c.btt.items()), {"parent": tok, "tree": tree})
        n = c.n
        cur = {k: list(c.cur[k]) for k in COLUMNS}
        # bpe.py:388 re-assigns the glue columns (float64), except with glue opt (bpe.py:381)
        cur_dt = {k: (np.float64 if k in GLUE and not glue_opt else object) for k in COLUMNS}
        idxes = sum([[i, i, i] for i in range(1, n + 1)], [])
        tok.__dict__.update({
            "_angles_and_dists": R._frame(pd, cur, cur_dt),
            "_angles_and_dists_orig": R._frame(pd, {k: list(c.orig[k]) for k in COLUMNS}, {k: object for k in COLUMNS}),
            "_coords": None, "beta_coords": None, "_idxes": idxes,
            "_res_idx_map": dict(zip(idxes[0::3], range(0, len(idxes), 3))), "_full_coords": None,
            "compute_sec_structs": False, "_sec": None, "_side_chains": None, "aa": None, "fname": c.fname,
            "n": n, "bond_labels": sum([[0, 1, 2] for _ in range(n - 1)] + [[0, 1]], []),
            "atom_labels": np.tile([0, 1, 2], n), "edges": [[j, j + 1, 0] for j in range(1, 3 * n)],
            "_bond_to_token": hier, "_init_n_ca": c.init[0], "_init_ca_c": c.init[1],
            "_init_bond_angle": c.init[2], "token_pos": list(c.token_pos), "tokens": list(c.tokens0),
        })
        if frames is not None:
            tok.__dict__["cached_all_frames"] = (list(frames[0]), list(frames[1]))
        return tok

    def _bpe_record(self, toks, C):
        import torch
        from sortedcontainers import SortedDict

        from . import refpickle as R
        sizes = sorted(k for k in self.bins)
        thr = R._new_dict(C["ThresholdDict"], [(k, v) for k, v in self._thresholds.items()], {"_int_keys": sizes})
        counts = self._bin_count_values()
        mk = lambda items: R._new_dict(C["ThresholdDict"], items, {"_int_keys": sizes})  # noqa: E731
        bin_counts = mk([(s0, counts[s0]) for s0 in sizes])
        centers = mk([(s0, {k: torch.tensor(v, dtype=torch.float32).mean(axis=-1)
                            for k, v in self._grid_only(s0).items()}) for s0 in sizes])
        weights = mk([(s0, {k: torch.tensor(v, dtype=torch.float32) / sum(v) for k, v in counts[s0].items()})
                      for s0 in sizes])
        nump = self.num_partitions
        if isinstance(nump, dict):
            nump = R._new_dict(C["ThresholdDict"], list(dict.items(nump)),
                               {"_int_keys": sorted(k for k in nump if isinstance(k, int))})
        attrs = {
            "tokenizers": toks, "compute_sec_structs": self.compute_sec_structs,
            "plot_iou_with_sec_structs": self.plot_iou_with_sec_structs,
            "rmsd_partition_min_size": self.rmsd_partition_min_size, "rmsd_super_res": self.rmsd_super_res,
            "rmsd_only": self.rmsd_only, "glue_opt": self.glue_opt, "glue_opt_every": self.glue_opt_every,
            "glue_opt_prior": self.glue_opt_prior, "glue_opt_method": self.glue_opt_method, "num_partitions": nump,
            "max_num_strucs": self.max_num_strucs, "res_init": self.res_init, "std_bonds": self.std_bonds,
            "bins": dict(self.bins), "bin_strategy": self.bin_strategy, "n": self.n, "seed": self.seed,
            "rng": self.rng, "save_dir": self.save_dir, "_step": self._step, "_times": list(self._times),
            "_ious": [], "_thresholds": thr, "_bin_counts": bin_counts, "_bin_centers": centers,
            "_bin_weights": weights, "_tokens": dict(self._tokens),
        }
        if hasattr(self, "_sphere_dict"):
            attrs["_sphere_dict"] = self._sphere_dict
        if hasattr(self, "_geo_dict"):
            attrs.update({"_geo_dict": self._geo_dict, "_priority_dict": SortedDict({p: None for p in self._priority}),
                          "_key_to_priority": self._key_to_priority, "_geo_step": self._geo_step,
                          "_sphere_keys": {}})
        return R._new(C["BPE"], attrs)

    @classmethod
    def from_checkpoint(cls, obj, device: int = 0, group=None):
        """The trained state tokenize() needs, from a checkpoint of this mode (this build's or
        the reference's, read by geobpe.refpickle.load): settings, _thresholds, _tokens,
        _sphere_dict.  bin/induce.py's RMSD-mode path.  ``group`` as in the constructor (the
        assignment batches split over the ranks); every attribute __init__ sets is set here too
        (tests/test_rmsd_mode.py compares the two)."""
        from .bpe import ThresholdDict
        self = cls.__new__(cls)
        self.device = int(device)
        self._group = _RmsdGroup(group, self.device) if group is not None else None
        self.bins = dict(obj.bins)
        self.B = int(self.bins[1])
        for k in ("bin_strategy", "res_init", "std_bonds", "rmsd_partition_min_size", "rmsd_super_res",
                  "rmsd_only", "glue_opt", "glue_opt_method", "glue_opt_every", "glue_opt_prior",
                  "max_num_strucs", "seed", "save_dir", "compute_sec_structs", "plot_iou_with_sec_structs"):
            setattr(self, k, getattr(obj, k, None))
        self.rmsd_super_res = bool(self.rmsd_super_res)
        self.std_bonds = True if self.std_bonds is None else bool(self.std_bonds)
        if self.glue_opt:  # the prior tables from the checkpoint's _bin_centers / _bin_weights
            from .glue import GLUE

            def arr(v):
                return np.asarray(v.numpy() if hasattr(v, "numpy") else v, dtype=np.float32)
            sizes = sorted(self.bins)
            kmax = max(len(arr(dict.__getitem__(obj._bin_centers, s0)[k])) for s0 in sizes for k in GLUE)
            table = np.zeros((len(sizes), 3, 2, kmax), dtype=np.float32)
            counts = np.zeros((len(sizes), 3), dtype=np.int32)
            for gi, s0 in enumerate(sizes):
                for t, k in enumerate(GLUE):
                    c = arr(dict.__getitem__(obj._bin_centers, s0)[k])
                    w = arr(dict.__getitem__(obj._bin_weights, s0)[k])
                    table[gi, t, 0, :len(c)], table[gi, t, 1, :len(w)], counts[gi, t] = c, w, len(c)
            self._glue_prior = (table, counts)
        thr = ThresholdDict()
        for k, v in dict.items(obj._thresholds):
            thr[k] = v
        self._thresholds = thr
        self._thr_by_len = {}
        self._key_edges = {}
        self._tokens = dict(obj._tokens)
        self._sphere_dict = dict(obj._sphere_dict)
        self.num_partitions = getattr(obj, "num_partitions", 3)
        self.assign_calls = 0
        self._chains, self._times, self._merge_log, self._step = [], [], [], int(getattr(obj, "_step", 0))
        self._ious = list(getattr(obj, "_ious", []) or [])
        self._corpus, self._fnames, self.n = None, None, 0  # (no training corpus: tokenize() brings chains)
        rng = getattr(obj, "rng", None)  # (the checkpoint's Generator in its saved state, else a fresh one)
        self.rng = rng if isinstance(rng, np.random.Generator) else np.random.default_rng(self.seed)
        return self

    def _grid_only(self, size):
        return {k: v for k, v in self._thresholds[size].items()}

    def _bin_count_values(self):
        """_bin_counts per grid (bpe.py:841-867): np.histogram counts of the values the
        thresholds came from (angles wrapped to [0, 2pi), tau with every chain's init angle;
        bond lengths too with free bonds)."""
        ro = self._corpus["row_off"]
        n_ca, ca_c, tau0 = _rmsd.init_geometry()
        keys = BOND_ANGLES + DIHEDRALS + ([] if self.std_bonds else BOND_TYPES)
        vals = {}
        for k in keys:
            col = np.asarray(self._corpus[k], dtype=np.float64)
            v = col[np.nan_to_num(col, nan=0.0) != 0.0]
            extra = {"tau": tau0, "N:CA": n_ca, "CA:C": ca_c}.get(k)
            if extra is not None:
                v = np.concatenate([v, np.full(len(ro) - 1, extra)])
            vals[k] = v if k in BOND_TYPES else (v + TWO_PI) % TWO_PI
        out = {}
        for s0, b in self.bins.items():
            out[s0] = {}
            for k in keys:
                if self.bin_strategy.startswith("histogram"):
                    rng_ = (0, TWO_PI) if "cover" in self.bin_strategy and k not in BOND_TYPES else None
                    cnt = np.histogram(vals[k], bins=int(b), range=rng_)[0]
                else:
                    edges = [a for a, _ in self._thresholds[s0][k]] + [self._thresholds[s0][k][-1][1]]
                    cnt = np.histogram(vals[k], bins=np.array(edges))[0]
                out[s0][k] = [np.int64(x) for x in cnt]
        return out

    def save_checkpoint(self, path: str) -> None:
        """``bpe_iter=t.pkl`` in the reference's format (bin/encode.py:427), written atomically
        (with a process group by rank 0 only: every rank holds the same state)."""
        import os

        from . import refpickle as R
        g = self._group
        if g is None or g.rank == 0:
            tmp = path + ".tmp"
            with open(tmp, "wb") as f:
                R.dump(self.checkpoint_object(), f)
            os.replace(tmp, path)
        if g is not None:  # (no rank returns before the file is there)
            g.barrier()

    def geometry(self):
        """Every chain's current 9 columns, concatenated (the reference's DataFrames)."""
        return {c: np.concatenate([np.asarray(ch.cur[c], dtype=np.float64) for ch in self._chains]) for c in COLUMNS}

    def visualize(self, key, output_path):
        return None

    def plot_times(self, output_path):
        return None

    def close(self):
        return None
