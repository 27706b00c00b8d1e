"""Host mirror of the reference's GeoBPE object API on the MI355X engine.

``geobpe.bpe.BPE`` has the constructor, methods and state attributes of
``foldingdiff.bpe.BPE`` (foldingdiff/bpe.py:33-88) that the scoped pure-histogram
mode uses, so a caller of the reference (bin/encode.py, train.py) can switch:

  reference                              here
  BPE(structures, bins, ...)             BPE(structures, bins, ...)   (+ device=, max_vocab=)
  bpe.initialize(path=None)              bpe.initialize()             bpe.py:91-103
  bpe.bin()                              bpe.bin()                    bpe.py:1431-1474
  bpe.step()                             bpe.step()                   bpe.py:1792-2166
  bpe.quantize(t | [t] | tuples)         bpe.quantize(...)            bpe.py:918-956
  bpe.dequantize / recover               same                         bpe.py:959-1002
  bpe.vocab_size / cum_bin_count(key)    same                         bpe.py:878-915
  bpe.capacity(tokenizer=False)          same                         bpe.py:885-902
  bpe._tokens / _thresholds / _step      same contents
  bpe.tokenizers[i].bond_to_token, .token_pos, .tokens, .tokenize(), .n

Scope: res_init=True, rmsd_partition_min_size=inf (no RMSD
partitioning), glue_opt=False, std_bonds=True, bins={1: B},
bin_strategy "histogram", "histogram-cover" or "uniform".  Any other configuration raises
NotImplementedError up front (the reference would run its float-geometry RMSD /
LBFGS paths there).

``run(n)`` is the fast path: n merges back to back on the device with no host
synchronisation in between (``step()`` synchronises once per merge, like the
reference's Python loop does by construction).
"""
from __future__ import annotations

import json
import time

import numpy as np

from .engine import ANGLE_TYPES, GeoBPEEngine
from .synth import COLUMNS

BOND_TYPES = ["N:CA", "CA:C", "0C:1N"]            # Tokenizer.BOND_TYPES (tokenizer.py:19)
BOND_ANGLES = ["tau", "CA:C:1N", "C:1N:1CA"]      # tokenizer.py:21
DIHEDRAL_ANGLES = ["psi", "omega", "phi"]          # tokenizer.py:22
BOND_LENGTHS = [1.46, 1.54, 1.34]                  # nerf.py:17-19 (N_CA, CA_C, C_N)
GLUE_KEYS = ["omega", "phi", "C:1N:1CA"]           # the res_init glue angles (bpe.py:381-391)


def num_bonds(geo: dict) -> int:
    """Tokenizer.num_bonds (tokenizer.py:299-301)."""
    return len(geo.get("N:CA", [])) + len(geo.get("CA:C", [])) + len(geo.get("0C:1N", []))


def structures_to_corpus(structures) -> dict:
    """Reference structure dicts (``{"angles": DataFrame, ...}``, the
    canonical_distances_and_dihedrals layout) -> one concatenated corpus."""
    cols = {c: [] for c in COLUMNS}
    lengths = []
    for s in structures:
        ang = s["angles"] if isinstance(s, dict) and "angles" in s else s
        n = None
        for c in COLUMNS:
            v = np.asarray(ang[c], dtype=np.float64)
            n = len(v) if n is None else n
            if len(v) != n:
                raise ValueError(f"column {c} has {len(v)} rows, expected {n}")
            cols[c].append(v)
        lengths.append(n)
    out = {c: (np.concatenate(v) if v else np.zeros(0)) for c, v in cols.items()}
    ro = np.zeros(len(lengths) + 1, dtype=np.int64)
    np.cumsum(lengths, out=ro[1:])
    out["row_off"] = ro
    return out


class ThresholdDict(dict):
    """int-key floor lookup (data_structures.py:264-296): size -> bin grid."""

    def __getitem__(self, key):
        if key in self.keys():
            return super().__getitem__(key)
        if isinstance(key, int):
            ks = sorted(k for k in self.keys() if isinstance(k, int))
            lo = [k for k in ks if k <= key]
            if lo:
                return super().__getitem__(lo[-1])
        raise KeyError(key)


class Tokenizer:
    """Read-only view of one chain's segmentation (foldingdiff/tokenizer.py):
    ``bond_to_token`` {start bond: (start bond, token id, #bonds)} in positional
    order, ``token_pos``, ``tokens``, ``tokenize()``."""
    BOND_TYPES = BOND_TYPES
    BOND_ANGLES = BOND_ANGLES
    DIHEDRAL_ANGLES = DIHEDRAL_ANGLES
    BOND_LENGTHS = BOND_LENGTHS
    num_bonds = staticmethod(num_bonds)

    def __init__(self, bpe: "BPE", row: int, n: int, starts: np.ndarray, ids: np.ndarray, enc: np.ndarray, fname=None):
        self._bpe = bpe
        self.row = row
        self.n = int(n)
        self.fname = fname
        self._starts = starts
        self._ids = ids
        self._enc = enc

    @property
    def tokens(self):
        out = []
        for k, (s, t) in enumerate(zip(self._starts, self._ids)):
            e = self._starts[k + 1] if k + 1 < len(self._starts) else self.n
            nb = 3 * (e - s) - (1 if e == self.n else 0)
            out.append((3 * int(s), int(t), int(nb)))
        return out

    @property
    def bond_to_token(self):
        return {t[0]: t for t in self.tokens}

    @property
    def token_pos(self):
        pos = []
        for s, _, nb in self.tokens:
            pos.extend([s] * nb)
        return pos

    def compute_coords(self, index=0, length=float("inf"), orig=False):
        """Tokenizer.compute_coords (tokenizer.py:347-363): NeRF (on the device) of the
        chain's geometry -- every value the run reads at its bin centre and the standard
        bond lengths (the frame a scoped run leaves, geobpe.refpickle.chain_frames), or the
        input values with orig=True (the init lengths / angle are the run's in both)."""
        import pandas as pd

        from . import refpickle, rmsd
        b = self._bpe
        corpus = b._global_corpus if b._global_corpus is not None else b._corpus
        ro = corpus["row_off"]
        cols = {c: np.asarray(corpus[c][ro[self.row]:ro[self.row + 1]], dtype=np.float64) for c in COLUMNS}
        thr1 = {k: [tuple(p) for p in v] for k, v in b._thresholds[1].items()}
        q, o = refpickle.chain_frames(pd, cols, thr1)
        frame = o if orig else q
        tau = thr1["tau"]
        from .engine import init_bond_angle
        init = (BOND_LENGTHS[0], BOND_LENGTHS[1],
                sum(tau[get_ind((init_bond_angle() + 2 * np.pi) % (2 * np.pi), tau)]) / 2)
        ln = min(length, 3 * self.n - 1 - index)
        return rmsd.compute_coords({c: frame[c].tolist() for c in COLUMNS}, [(index, int(ln))], init=init,
                                   device=b._engine.device)[0]

    def tokenize(self):
        """tokenizer.py:379-392: MOTIF ids and the glue values (bin centres) after
        every token but the last."""
        thr = self._bpe._thresholds[1]
        K = len(self._bpe._tokens)
        B = self._bpe.B
        out = []
        enc = self._enc
        for k, t in enumerate(self._ids):
            out.append(("MOTIF", int(t)))
            if k + 1 < len(self._ids):
                om, ph, cn = (int(x) for x in enc[4 * k + 1: 4 * k + 4])
                out.append(("DIHEDRAL", "omega", sum(thr["omega"][om - K - B]) / 2))
                out.append(("DIHEDRAL", "phi", sum(thr["phi"][ph - K - 2 * B]) / 2))
                out.append(("BOND_ANGLE", "C:1N:1CA", sum(thr["C:1N:1CA"][cn - K]) / 2))
        return out


def _check_scope(bins, bin_strategy, res_init, std_bonds, rmsd_partition_min_size, glue_opt, compute_sec_structs):
    if not isinstance(bins, dict) or 1 not in bins:
        raise KeyError("bins must be a dict with key 1 (quantize/capacity need bins[1], bpe.py:896,909,952)")
    if len(bins) != 1:
        # the reference's step computes the new neighbour keys (bpe.py:1990-2006) before it
        # re-snaps the merged span to grid(|token|) (bpe.py:2010-2013): with several grids the
        # stored keys go stale and step() reaches breakpoint() at bpe.py:1917-1920
        # (tests/golden/multigrid_reference.json)
        # (BPE(...) hands such schedules to the host mirror, geobpe.rmsd_bpe; this is the
        # device engine's own guard)
        raise NotImplementedError("multi-grid bin schedules (--bins 1-a:s-b): the reference's step() is inconsistent "
                                  "for them (stale neighbour keys -> breakpoint at bpe.py:1919); see DESIGN.md §7")
    if bin_strategy not in ("histogram", "histogram-cover", "uniform"):
        raise NotImplementedError(f"bin_strategy={bin_strategy!r} (histogram / histogram-cover / uniform)")
    if not res_init:
        raise NotImplementedError("res_init=False cannot quantize in the reference either (SURVEY App. A)")
    if not std_bonds:
        # the reference's res_init quant_geo bins bond lengths through _thresholds[bond]
        # (bpe.py:1518-1519), which only std_bonds creates (bpe.py:874-876): its
        # initialize() raises KeyError('N:CA') (tests/golden/multigrid_reference.json,
        # "free-bonds"); this build raises the same error before any device work
        raise KeyError("N:CA")
    if rmsd_partition_min_size != float("inf") and rmsd_partition_min_size < 10 ** 9:
        raise NotImplementedError("RMSD partitioning (p_min_size < inf) is float geometry, SURVEY §8(f) row 4")
    if glue_opt:
        raise NotImplementedError("glue optimisation without RMSD partitioning: the reference re-optimises "
                                  "glues only after RMSD-key merges (bpe.py:2027); run it with a finite "
                                  "rmsd_partition_min_size (geobpe.rmsd_bpe.RmsdBPE)")
    if compute_sec_structs:
        raise NotImplementedError("secondary-structure priorities are not in this build")


class BPE:
    def __new__(cls, *args, **kwargs):
        """A finite rmsd_partition_min_size (the reference's default is 4) selects the
        RMSD-partitioned mode, geobpe.rmsd_bpe.RmsdBPE; so do a multi-grid
        schedule and bond-level init (res_init=False)."""
        if cls is BPE:
            import inspect
            ba = inspect.signature(BPE.__init__).bind(None, *args, **kwargs)
            ba.apply_defaults()
            p = ba.arguments["rmsd_partition_min_size"]
            bins = ba.arguments["bins"]
            if (p != float("inf") and p < 10 ** 9) or (isinstance(bins, dict) and len(bins) > 1 and 1 in bins) \
                    or not ba.arguments["res_init"]:
                # the host mirror: RMSD partitioning, a multi-grid schedule without it (the
                # reference's stale-key semantics), or bond-level init (res_init=False,
                # bpe.py:397-420); the device engine runs bins={1: B} from residue tokens
                from .rmsd_bpe import RmsdBPE
                return RmsdBPE(*args, **kwargs)
        return super().__new__(cls)

    def __init__(self, structures, bins, bin_strategy="histogram", save_dir="./plots/bpe",
                 compute_sec_structs=False, plot_iou_with_sec_structs=False, res_init=False, std_bonds=True,
                 rmsd_partition_min_size=4, rmsd_super_res=False, rmsd_only=False, num_partitions=3,
                 max_num_strucs=500, glue_opt=False, glue_opt_prior=0.0, glue_opt_every=10,
                 glue_opt_method="all", seed=None, device: int = 0, max_vocab: int = 1 << 20, group=None,
                 record_tree: bool = True, global_corpus=None):
        """``group`` (geobpe.dist.TorchGroup): this process holds one row shard
        (``structures``) of a multi-GPU run; ``global_corpus`` (the whole corpus,
        needed on rank 0 for checkpoints) -- encode_all / capacity / checkpoints
        then gather every rank's chains to rank 0 (None on the other ranks)."""
        _check_scope(bins, bin_strategy, res_init, std_bonds, rmsd_partition_min_size, glue_opt, compute_sec_structs)
        if isinstance(structures, dict) and "row_off" in structures:
            corpus = structures
            self._fnames = list(structures["fnames"]) if structures.get("fnames") is not None else None
        else:
            structures = list(structures)
            corpus = structures_to_corpus(structures)
            self._fnames = [s.get("fname") if isinstance(s, dict) else None for s in structures]
        self._corpus = corpus
        self.bins = bins
        self.B = int(bins[1])
        self.bin_strategy = bin_strategy
        self.save_dir = save_dir
        self.compute_sec_structs = compute_sec_structs
        self.plot_iou_with_sec_structs = plot_iou_with_sec_structs
        self.res_init = res_init
        self.std_bonds = std_bonds
        self.rmsd_partition_min_size = rmsd_partition_min_size
        self.rmsd_super_res = rmsd_super_res
        self.rmsd_only = rmsd_only
        self.num_partitions = num_partitions
        self.max_num_strucs = max_num_strucs
        self.glue_opt = glue_opt
        self.glue_opt_prior = glue_opt_prior
        self.glue_opt_every = glue_opt_every
        self.glue_opt_method = glue_opt_method
        self.seed = seed
        self.rng = np.random.default_rng(seed)
        self.n = len(corpus["row_off"]) - 1
        self._step = 0
        self._times = []
        self._ious = []
        self._tokens = {}
        self._engine = GeoBPEEngine(corpus, self.B, device=device, max_vocab=max_vocab, group=group,
                                    strategy=bin_strategy)
        self._tok_cache = None
        self._record_tree = bool(record_tree)
        self._group = group
        self._global_corpus = global_corpus

    # ------------------------------------------------------------ BPE.initialize
    def initialize(self, path=None):
        e = self._engine
        e.initialize()
        thr = ThresholdDict()
        thr[1] = {k: list(v) for k, v in e.thresholds.items()}
        for i, bt in enumerate(BOND_TYPES):  # std_bonds (bpe.py:874-876)
            thr[bt] = [(BOND_LENGTHS[i], BOND_LENGTHS[i])]
        self._thresholds = thr
        self._tokens = {v: self._residue_token(int(s)) for v, s in enumerate(e.sym_of_label)}
        self._tok_cache = None
        return self

    def _residue_token(self, sym: int) -> dict:
        """_tokens[label] of a residue token: its bin-centre geometry (bpe.py:236-261)."""
        B = self.B
        thr = self._thresholds[1]
        c = lambda k, i: sum(thr[k][i]) / 2  # noqa: E731  (bpe.py:1509)
        if sym >= B ** 3:
            d = {"N:CA": [1.46], "CA:C": [1.54], "tau": [c("tau", sym - B ** 3)]}
        else:
            d = {"N:CA": [1.46], "CA:C": [1.54], "0C:1N": [1.34], "tau": [c("tau", sym // (B * B))],
                 "CA:C:1N": [c("CA:C:1N", sym // B % B)], "psi": [c("psi", sym % B)]}
        return dict(sorted(d.items()))  # the reference keeps json.dumps(sort_keys=True) order

    @property
    def _bin_counts(self):
        """np.histogram counts per grid-1 type (bpe.py:864-866), computed on demand."""
        out = ThresholdDict()
        counts = {}
        corpus = self._global_corpus if self._global_corpus is not None else self._corpus
        ro = corpus["row_off"]
        from .engine import init_bond_angle
        for key in ANGLE_TYPES:
            col = np.asarray(corpus[key])
            vals = col[np.nan_to_num(col, nan=0.0) != 0.0]
            if key == "tau":
                vals = np.concatenate([vals, np.full(len(ro) - 1, init_bond_angle())])
            a = (vals + 2 * np.pi) % (2 * np.pi)
            edges = [s for s, _ in self._thresholds[1][key]] + [self._thresholds[1][key][-1][1]]
            counts[key] = list(np.histogram(a, bins=np.array(edges))[0])
        out[1] = counts
        return out

    # ------------------------------------------------------------ bin / step
    def bin(self):
        self._engine.bin()
        if self._record_tree:  # merge events for the checkpoint's merge tree (refpickle)
            self._engine.record_events(True)
        self._tok_cache = None

    def step(self):
        t0 = time.time()
        r = self._engine.step()
        if r is None:
            raise IndexError("no token pair left to merge")  # SortedDict.peekitem(0) on an empty dict
        nid = r[0]
        self._tokens[nid] = json.loads(self._engine.token_json(nid))  # bpe.py:1857-1860
        self._step += 1
        self._times.append(time.time() - t0)
        self._tok_cache = None

    def run(self, n_merges: int) -> int:
        """n merges back to back on the device (no host sync between them)."""
        t0 = time.time()
        done = self._engine.run(n_merges)
        k0 = len(self._tokens)
        for nid, _, _ in self._engine.merges[k0 - self._engine.K0:]:
            self._tokens[nid] = json.loads(self._engine.token_json(nid))
        self._step += done
        if done:
            self._times.extend([(time.time() - t0) / done] * done)
        self._tok_cache = None
        return done

    @property
    def merges(self):
        """[(key string, count)] -- the merge list."""
        return self._engine.merge_keys()

    # ------------------------------------------------------------ vocab / encode
    @property
    def vocab_size(self):
        return len(self._tokens) + self.cum_bin_count()

    def cum_bin_count(self, key=None):
        """bpe.py:905-915 (res_init: only the glue types count)."""
        if self.res_init:
            assert key is None or key in GLUE_KEYS
        count = 0
        for k in ANGLE_TYPES:  # _bin_counts[1] key order
            if key == k:
                break
            if self.res_init and k not in GLUE_KEYS:
                continue
            count += self.B
        return count

    @property
    def tokenizers(self):
        if self._tok_cache is None:
            start, ids, off = self._engine.segmentation()
            enc, eoff = self._engine.encode()
            ro = self._corpus["row_off"]
            toks = []
            for r in range(self.n):
                toks.append(Tokenizer(self, r, int(ro[r + 1] - ro[r]), start[off[r]:off[r + 1]],
                                      ids[off[r]:off[r + 1]], enc[eoff[r]:eoff[r + 1]],
                                      fname=self._fnames[r] if self._fnames else None))
            self._tok_cache = (toks, enc, eoff)
        return self._tok_cache[0]

    def _gather(self, part: dict):
        """Every rank's ``part`` on rank 0 (rank order), None elsewhere; [part] alone."""
        g = self._group
        if g is None:
            return [part]
        parts = [None] * g.world_size if g.rank == 0 else None
        g.dist.gather_object(part, parts, dst=0, group=g.pg)
        return parts

    @staticmethod
    def _cat_offsets(offs):
        out = [np.zeros(1, dtype=np.int64)]
        base = 0
        for o in offs:
            out.append(np.asarray(o[1:], dtype=np.int64) + base)
            base += int(o[-1])
        return np.concatenate(out)

    @staticmethod
    def _merge_rank_events(parts):
        """Every rank's merge events (rank-local slots, merge t's in [eoff[t],
        eoff[t+1])) as global slots (+ the rank's residue base), merge by merge in
        rank order -- ascending slot within a merge, as a 1-GPU run logs them."""
        M = len(parts[0]["eoff"]) - 1
        t = np.concatenate([np.repeat(np.arange(M), np.diff(p["eoff"])) for p in parts])
        ga = np.concatenate([np.asarray(p["a"], np.int64) + p["base"] for p in parts])
        gb = np.concatenate([np.asarray(p["b"], np.int64) + p["base"] for p in parts])
        order = np.argsort(t, kind="stable")
        return ga[order], gb[order], np.searchsorted(t[order], np.arange(M + 1), side="left").astype(np.int64)

    def encode_all(self):
        """quantize(tokenize()) of every chain as (ids, row offsets), one device pass
        (multi-GPU: every rank's chains in global order on rank 0, None elsewhere)."""
        ids, off = self._engine.encode()
        if self._group is None:
            return ids, off
        parts = self._gather({"ids": ids, "off": off})
        if parts is None:
            return None
        return np.concatenate([p["ids"] for p in parts]), self._cat_offsets([p["off"] for p in parts])

    def quantize(self, tokenized):
        """bpe.py:918-956: a Tokenizer, a list of Tokenizers (one device encode
        pass for all) or a list of token tuples."""
        if isinstance(tokenized, Tokenizer):
            return [int(x) for x in tokenized._enc]
        if len(tokenized) and isinstance(tokenized[0], Tokenizer):
            return [[int(x) for x in t._enc] for t in tokenized]
        return self._quantize_tuples(tokenized)

    def _quantize_tuples(self, tokenized):
        K = len(self._tokens)
        ids = list(self._tokens)
        out = []
        for tok in tokenized:
            if tok[0] == "MOTIF":
                out.append(ids.index(tok[1]))
            else:
                dt = tok[1]
                relv = self._thresholds[1][dt]
                out.append(K + self.cum_bin_count(dt) + get_ind((tok[2] + 2 * np.pi) % (2 * np.pi), relv))
        return out

    def dequantize(self, quantized):
        """bpe.py:959-983."""
        cum = self.cum_bin_count()
        nv = self.vocab_size
        out = []
        for i, q in enumerate(quantized):
            if q < nv - cum:
                if q > len(self._tokens):
                    raise ValueError(f"pos {i} > vocab range=(0, {len(self._tokens)})")
                out.append(("MOTIF", list(self._tokens)[q]))
            else:
                c = q - (nv - cum)
                tok = None
                for k in ANGLE_TYPES:
                    if self.res_init and k not in GLUE_KEYS:
                        continue
                    v = self._thresholds[1][k]
                    if c < len(v):
                        s, e = v[c]
                        tok = ("DIHEDRAL" if k in DIHEDRAL_ANGLES else "BOND_ANGLE", k, (s + e) / 2)
                        break
                    c -= len(v)
                if tok is None:
                    raise ValueError(f"pos {i} > vocab_size={nv}")
                out.append(tok)
        return out

    def recover(self, tokenized):
        """bpe.py:986-1002."""
        from collections import defaultdict
        repl = defaultdict(list)
        for tok in tokenized:
            if tok[0] == "MOTIF":
                kd = self._tokens[tok[1]]
                for k in kd:
                    repl[k] += kd[k]
            else:
                repl[tok[1]].append(tok[2])
        return dict(repl)

    @staticmethod
    def init_structure(n):
        """bpe.py:1005-1027."""
        from .rmsd_bpe import init_structure
        return init_structure(n)

    def recover_structure(self, repl, tokenized):
        """bpe.py:1029-1051 (bin/train.py:715-716): a tokenizer (chain view with
        bond_to_token, token_geo, tokenize, compute_coords) built from recovered geometry."""
        from .rmsd_bpe import recover_structure
        return recover_structure(self._tokens, repl, tokenized, self._engine.device)

    def capacity(self, tokenizer=False):
        """bpe.py:885-902."""
        total = 0
        for token in self._tokens.values():
            n = num_bonds(token)
            total += 4 * (n + n - 1 + n - 2) * 8
        if tokenizer:
            mbits = np.log2(len(self._tokens))
            bbits = np.log2(self.bins[1])
            enc = self.encode_all()
            if enc is None:  # multi-GPU: rank 0 answers
                return None
            eoff = enc[1]
            for L in np.diff(eoff):
                m = (int(L) + 3) // 4
                total += mbits * m
                total += 3 * (m - 1) * bbits
        return total

    # ------------------------------------------------------------ checkpoints
    def checkpoint_state(self) -> dict:
        """The run state geobpe.refpickle turns into the reference's BPE object."""
        if not self._record_tree:
            raise RuntimeError("checkpoints need record_tree=True (the merge tree)")
        e = self._engine
        start, ids, off = e.segmentation()
        a, b, eoff = e.events()
        corpus, fnames = self._corpus, self._fnames
        if self._group is not None:  # every rank's chains and merge events, in global order, on rank 0
            parts = self._gather({"start": start, "ids": ids, "off": off, "a": a, "b": b, "eoff": eoff,
                                  "base": self._group.residue_base})
            if parts is None:
                return None
            if self._global_corpus is None:
                raise RuntimeError("multi-GPU checkpoints need global_corpus on rank 0")
            start = np.concatenate([p["start"] for p in parts])
            ids = np.concatenate([p["ids"] for p in parts])
            off = self._cat_offsets([p["off"] for p in parts])
            a, b, eoff = self._merge_rank_events(parts)
            corpus = self._global_corpus
            fnames = list(corpus["fnames"]) if corpus.get("fnames") is not None else None
        ro = corpus["row_off"]
        return {
            "corpus": corpus, "fnames": fnames or [None] * (len(ro) - 1),
            "B": self.B, "bins": dict(self.bins), "bin_strategy": self.bin_strategy,
            "thresholds": {k: list(v) for k, v in self._thresholds[1].items()},
            "bin_counts": self._bin_counts[1], "K0": e.K0, "tokens": dict(self._tokens),
            "seg_start": start, "seg_id": ids, "seg_off": off, "ev_a": a, "ev_b": b, "ev_off": eoff,
            "step": self._step, "times": list(self._times),
            "args": {k: getattr(self, k) for k in ("compute_sec_structs", "plot_iou_with_sec_structs",
                                                  "rmsd_partition_min_size", "rmsd_super_res", "rmsd_only",
                                                  "glue_opt", "glue_opt_every", "glue_opt_prior", "glue_opt_method",
                                                  "num_partitions", "max_num_strucs", "seed", "save_dir")},
        }

    def save_checkpoint(self, path: str) -> None:
        """``bpe_iter=t.pkl`` in the reference's format (bin/encode.py:427): a
        pickle of foldingdiff.bpe.BPE that train.py / predict.py / induce.py and
        the reference's own resume load unchanged (geobpe.refpickle)."""
        from . import refpickle
        state = self.checkpoint_state()  # (multi-GPU: every rank gathers, rank 0 writes)
        if state is not None:
            refpickle.save(state, path)

    def visualize(self, key, output_path):  # plotting only in the reference (bpe.py:1583-1627)
        return None

    def plot_times(self, output_path):
        return None

    def close(self):
        self._engine.close()


def get_ind(v, values):
    """BPE.get_ind (bpe.py:1164-1189)."""
    import bisect
    left = [s for s, _ in values]
    ind = bisect.bisect_right(left, v) - 1
    if ind < 0:
        raise ValueError(f"value {v} is below the first bin range")
    s, e = values[ind]
    if ind == len(values) - 1 and v == e:
        return ind
    if s <= v < e:
        return ind
    raise ValueError(f"value {v} does not fall into any bin")


def get_codebook_utility(input_ids, vocab_size, eps=1e-8):
    """plotting.py:78-95 (numpy restatement; used by the stats JSON)."""
    ids = np.asarray(input_ids, dtype=np.int64)
    cnt = np.bincount(ids, minlength=vocab_size).astype(np.float32)
    p = cnt / cnt.sum()
    ent = float(-np.sum(p * np.log(p + np.float32(eps)), dtype=np.float32))
    ppl = float(np.exp(np.float32(ent)))
    return {"perplexity": ppl, "perplexity_normalized": ppl / vocab_size, "entropy": ent,
            "entropy_normalized": ent / vocab_size, "use_ratio": float(np.count_nonzero(cnt) / len(cnt))}
