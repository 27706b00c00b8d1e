"""GeoBPEEngine: the host driver of libgeobpe.so for one corpus shard.

It runs the reference's scoped GeoBPE pipeline:

  initialize()   BPE._init_thresholds + BPE._init_res_tokens (bpe.py:820-876, 138-394):
                 device min/max of the wrapped angle columns -> np.histogram edges on
                 the host (exactly the reference's edges, plotting.py:305-337) ->
                 device quantisation of every residue / junction -> first-appearance
                 labels (bpe.py:236-246).
  bin()          BPE.bin (bpe.py:1431-1474) -- full content-keyed pair histogram.
  step()         BPE.step (bpe.py:1792-2166) -- one merge.
  encode()       quantize(tokenize()) for every chain (bpe.py:918-956).

Multi-GPU: each rank holds a contiguous block of chains (row sharding,
SURVEY.md §8(e)).  Thresholds and first appearances are all-reduced once;
then every iteration the ranks select the same winner from replicated global
counts, apply it locally and exchange their count deltas (one all-gather of
40-byte records of the keys whose local count changed).
"""
from __future__ import annotations

import ctypes
import math
from typing import Optional

import numpy as np

from . import _native
from .synth import COLUMNS

ANGLE_TYPES = ["tau", "CA:C:1N", "C:1N:1CA", "psi", "omega", "phi"]
TWO_PI = 2 * np.pi
# nerf.py:22-24 -- Tokenizer._init_bond_angle (tokenizer.py:74-77, angles_and_coords.py:746-752)
_N_INIT = np.array([17.047, 14.099, 3.625])
_CA_INIT = np.array([16.967, 12.784, 4.338])
_C_INIT = np.array([15.685, 12.755, 5.133])


def init_bond_angle() -> float:
    v1, v2 = _N_INIT - _CA_INIT, _C_INIT - _CA_INIT
    u1 = v1 / np.linalg.norm(v1)
    u2 = v2 / np.linalg.norm(v2)
    return float(np.arccos(np.clip(np.dot(u1, u2), -1.0, 1.0)))


def histogram_edges(mn: float, mx: float, count: int, B: int, cover: bool = False) -> np.ndarray:
    """np.histogram(a, bins=B) edges given only min/max/len of ``a`` (numpy's
    _get_outer_edges + linspace depend on nothing else).  ``cover``: the
    "histogram-cover" strategy, range=(0, 2*pi) (plotting.py:319)."""
    a = np.array([mn, mx], dtype=np.float64) if count > 0 else np.zeros(0, dtype=np.float64)
    return np.histogram_bin_edges(a, bins=B, range=(0, TWO_PI) if cover else None)


def equal_count_edges(col: np.ndarray, n_rows: int, key: str, B: int) -> np.ndarray:
    """bin_strategy "uniform": np.quantile of the sorted wrapped values at
    linspace(0, 1, B+1) (equal_count_bin_edges / save_histogram_equal_counts,
    plotting.py:256-302), over the values _init_thresholds collects (non-NaN,
    non-zero; tau + the init angle per chain, bpe.py:842-846).  An order
    statistic of the whole column: computed on the host copy of the input (the
    prologue; the histogram strategies need only the device min / max)."""
    vals = col[np.nan_to_num(col, nan=0.0) != 0.0]
    if key == "tau":
        vals = np.concatenate([vals, np.full(n_rows, init_bond_angle())])
    a = (vals + TWO_PI) % TWO_PI
    return np.quantile(np.sort(a), np.linspace(0, 1, B + 1))


def _p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def _stream_handle(device: int):
    try:
        import torch
        if torch.cuda.is_available():
            return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)
    except Exception:
        pass
    return None


class GeoBPEEngine:
    def __init__(self, corpus: dict, bins: int, device: int = 0, max_vocab: int = 1 << 20,
                 group=None, stream=None, use_torch_stream: bool = True, cover: bool = False,
                 bin_dense: bool = True, strategy: Optional[str] = None, tail: Optional[int] = None,
                 mid: Optional[int] = None, collapse: bool = True):
        """``corpus``: ``{column: float64[R]}`` + ``row_off`` (geobpe.synth layout) for
        THIS shard.  ``group``: an exchange group (geobpe.dist) for multi-rank runs.
        ``tail``: merges of at most this count run in the one-workgroup late-merge
        kernel (include/geobpe.h geobpe_set_tail; None = the library default, 0 = never);
        ``mid``: merges of at most this count run in the two-launch middle-regime kernels
        (geobpe_set_mid); ``collapse``: multi-rank runs stop sharding at that switch, every
        rank going on with the whole corpus (geobpe_set_collapse)."""
        self.L = _native.lib()
        self.B = int(bins)
        self.device = int(device)
        self.group = group
        self.cover = bool(cover)
        self.strategy = strategy or ("histogram-cover" if cover else "histogram")
        if self.strategy not in ("histogram", "histogram-cover", "uniform"):
            raise NotImplementedError(f"bin_strategy={self.strategy!r}")
        self.cover = self.strategy == "histogram-cover"
        self.bin_dense = bool(bin_dense)
        # multi-rank run(): the pipelined exchange (no host wait per merge, geobpe.dist)
        self.pipelined = True
        self._events_on = False
        self.row_off = np.ascontiguousarray(corpus["row_off"], dtype=np.int64)
        self.n_rows = len(self.row_off) - 1
        self._cols = [np.ascontiguousarray(corpus[c], dtype=np.float64) for c in COLUMNS]
        self.torch_stream = None
        if stream is None and group is not None and (getattr(group, "world_size", 1) > 1 or getattr(group, "force", False)):
            # multi-rank: the engine's kernels and the exchange's torch ops (copies,
            # collectives) must be ordered on ONE stream -- a torch stream of our own
            import torch
            self.torch_stream = torch.cuda.Stream(device=self.device)
            stream = ctypes.c_void_p(self.torch_stream.cuda_stream)
        if stream is None and use_torch_stream:
            stream = _stream_handle(self.device)
        self._ctx = ctypes.c_void_p()
        rc = self.L.geobpe_create(ctypes.byref(self._ctx), self.device, stream, int(max_vocab))
        if rc:
            msg = self.L.geobpe_last_error(self._ctx) if self._ctx else b"create failed"
            raise _native.GeoBPEError(f"geobpe_create: {msg.decode() if msg else rc}")
        if tail is not None:
            self._chk(self.L.geobpe_set_tail(self._ctx, int(tail)))
        if mid is not None:
            self._chk(self.L.geobpe_set_mid(self._ctx, int(mid)))
        self._chk(self.L.geobpe_set_collapse(self._ctx, 1 if collapse else 0))
        self._collapsed = False
        self.K0 = 0
        self.merges = []  # [(new_id, count, n_merged)]
        self.thresholds = None
        self._initialized = False
        self._binned = False
        self._delta_buf = None
        self._done = False

    # ------------------------------------------------------------ helpers
    def _chk(self, rc):
        _native.check(self._ctx, rc)

    @property
    def distributed(self) -> bool:
        """Row-sharded with an exchange per merge (until a collapse: then every rank holds the
        whole corpus and runs the one-rank loop)."""
        return (self.group is not None and (self.group.world_size > 1 or getattr(self.group, "force", False))
                and not self._collapsed)

    @property
    def collapsed(self) -> bool:
        return self._collapsed

    def close(self):
        if self._ctx:
            self.L.geobpe_destroy(self._ctx)
            self._ctx = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------ prologue
    def initialize(self, thresholds: Optional[dict] = None, sym_of_label=None):
        """Thresholds (bpe.py:820-876), residue symbols and first-appearance labels.
        ``thresholds`` ({type: [(start, end)]}) and ``sym_of_label`` fix a trained
        vocabulary's grid and residue labels instead (merge replay on new chains)."""
        arr = (ctypes.c_void_p * 9)(*[c.ctypes.data for c in self._cols])
        self._chk(self.L.geobpe_load_angles(self._ctx, self.n_rows, _p(self.row_off), arr))
        edges = np.zeros((6, self.B + 1), dtype=np.float64)
        if thresholds is not None:
            self.thresholds = {}
            for t, key in enumerate(ANGLE_TYPES):
                v = [(float(a), float(b)) for a, b in thresholds[key]]
                if len(v) != self.B:
                    raise ValueError(f"thresholds[{key!r}] has {len(v)} bins, expected {self.B}")
                edges[t] = [a for a, _ in v] + [v[-1][1]]
                self.thresholds[key] = v
        elif self.strategy == "uniform":
            if self.distributed:
                raise NotImplementedError("uniform bins need the global quantiles: single rank only")
            self.thresholds = {}
            for t, key in enumerate(ANGLE_TYPES):
                e = equal_count_edges(self._cols[COLUMNS.index(key)], self.n_rows, key, self.B)
                edges[t] = e
                self.thresholds[key] = [(float(s), float(f)) for s, f in zip(e[:-1], e[1:])]
        else:
            mm = np.zeros(12, dtype=np.float64)
            cnt = np.zeros(6, dtype=np.int64)
            self._chk(self.L.geobpe_angle_range(self._ctx, _p(mm), _p(cnt)))
            n_rows_total = self.n_rows
            if self.distributed:
                mm, cnt, n_rows_total = self.group.reduce_ranges(mm, cnt, self.n_rows)
            self._range_stats = (mm.copy(), cnt.copy(), n_rows_total)
            self.thresholds = {}
            for t, key in enumerate(ANGLE_TYPES):
                e = self._hist_edges(t, key, self.B)
                edges[t] = e
                self.thresholds[key] = [(float(s), float(f)) for s, f in zip(e[:-1], e[1:])]
        self._edges = edges
        self._chk(self.L.geobpe_quantize(self._ctx, self.B, _p(edges), init_bond_angle()))
        S = self.B ** 3 + self.B
        first = np.zeros(S, dtype=np.int64)
        row_base = 0 if not self.distributed else self.group.residue_base
        self._chk(self.L.geobpe_symbol_first(self._ctx, row_base, _p(first)))
        if self.distributed:
            first = self.group.reduce_first(first)
        present = np.nonzero(first != np.iinfo(np.int64).max)[0]
        label_of_sym = np.full(S, -1, dtype=np.int32)
        if sym_of_label is not None:
            order = np.asarray(sym_of_label, dtype=np.int64)
            label_of_sym[order] = np.arange(len(order), dtype=np.int32)
            unknown = present[label_of_sym[present] < 0]
            if len(unknown):
                raise ValueError(f"{len(unknown)} residue geometries (symbols {unknown[:5].tolist()}) are not in "
                                 "the trained vocabulary")
        else:
            order = present[np.argsort(first[present], kind="stable")]
            label_of_sym[order] = np.arange(len(order), dtype=np.int32)
        self.K0 = int(len(order))
        self.sym_of_label = order.astype(np.int32)
        self._chk(self.L.geobpe_init_tokens(self._ctx, _p(label_of_sym), self.K0))
        self._initialized = True
        return self

    def _hist_edges(self, t: int, key: str, B: int) -> np.ndarray:
        """np.histogram edges of angle type t with B bins from the device min / max /
        count (bpe.py:836-866; tau also holds every chain's init angle, :845-846)."""
        mm, cnt, n_rows_total = self._range_stats
        w0 = (init_bond_angle() + TWO_PI) % TWO_PI
        mn, mx, c = float(mm[2 * t]), float(mm[2 * t + 1]), int(cnt[t])
        if key == "tau" and n_rows_total > 0:
            mn, mx, c = (min(mn, w0), max(mx, w0), c + n_rows_total) if c > 0 else (w0, w0, n_rows_total)
        return histogram_edges(mn, mx, c, B, self.cover)

    def thresholds_for(self, B: int) -> dict:
        """Thresholds of another grid size's bin count over the same values (a multi-grid
        ``bins`` schedule: bpe.py:836-869 runs the same histogram per size)."""
        out = {}
        for t, key in enumerate(ANGLE_TYPES):
            if self.strategy == "uniform":
                e = equal_count_edges(self._cols[COLUMNS.index(key)], self.n_rows, key, int(B))
            else:
                e = self._hist_edges(t, key, int(B))
            out[key] = [(float(s), float(f)) for s, f in zip(e[:-1], e[1:])]
        return out

    def replay_load(self, rec: dict):
        """Merge replay: merge t becomes the trained token K0 + t (geobpe.induce
        builds ``rec``: h1, h2, len, idL, g, idR arrays)."""
        if not self._binned:
            raise RuntimeError("bin() first")
        h1 = np.ascontiguousarray(rec["h1"], dtype=np.uint64)
        h2 = np.ascontiguousarray(rec["h2"], dtype=np.uint64)
        ln, a, g, b = (np.ascontiguousarray(rec[k], dtype=np.int32) for k in ("len", "idL", "g", "idR"))
        self._chk(self.L.geobpe_replay_load(self._ctx, _p(h1), _p(h2), _p(ln), _p(a), _p(g), _p(b), len(h1)))
        self._replay_n = len(h1)

    # ------------------------------------------------------------ histogram / merges
    def bin(self):
        if not self._initialized:
            raise RuntimeError("initialize() first")
        if self.distributed:
            self._chk(self.L.geobpe_set_distributed(self._ctx, 1))
            self._chk(self.L.geobpe_set_global_residues(self._ctx, self.group.total_residues))
            self._chk(self.L.geobpe_set_rank(self._ctx, int(getattr(self.group, "rank", 0))))
        self._chk(self.L.geobpe_set_bin_dense(self._ctx, 1 if self.bin_dense else 0))
        self._chk(self.L.geobpe_bin(self._ctx))
        if self.distributed:
            self._exchange()
        self._binned = True

    def _exchange(self):
        """export local count deltas -> all-gather -> import on every rank."""
        n = ctypes.c_int64(0)
        cap, ptr = self.group.export_buffer(self)
        self._chk(self.L.geobpe_delta_export(self._ctx, ptr, cap, ctypes.byref(n)))
        d_in, total = self.group.all_gather_deltas(self, int(n.value))
        self._chk(self.L.geobpe_delta_import(self._ctx, d_in, total))

    def step(self, want_merged: bool = True):
        """One merge. Returns (new_id, count, n_merged) or None if no pair is left."""
        if not self._binned:
            raise RuntimeError("bin() first")
        nid, cnt = ctypes.c_int32(0), ctypes.c_int32(0)
        nm = ctypes.c_int64(0)
        if not self.distributed:
            self._chk(self.L.geobpe_step(self._ctx, ctypes.byref(nid), ctypes.byref(cnt), ctypes.byref(nm)))
            if nid.value < 0:
                self._done = True
                return None
        else:
            self._chk(self.L.geobpe_step_select(self._ctx, ctypes.byref(nid), ctypes.byref(cnt)))
            if nid.value < 0:
                self._done = True
                return None
            self._chk(self.L.geobpe_step_apply(self._ctx, ctypes.byref(nm) if want_merged else None))
            self.group.exchange_async(self)
        want = want_merged or not self.distributed
        rec = (int(nid.value), int(cnt.value), int(nm.value) if want else -1)
        self.merges.append(rec)
        return rec

    def run(self, n_merges: int) -> int:
        """Enqueue ``n_merges`` iterations with no host synchronisation in between
        (device-side argmax + tie-break); returns the merges actually made."""
        if not self._binned:
            raise RuntimeError("bin() first")
        if self.distributed:
            if self.pipelined and getattr(self.group, "engine_exchange", False) and hasattr(self.group, "attach"):
                # the engine's own N > 1 loop; the run's merge records come back with it
                self.group.attach(self)
                n, first = ctypes.c_int64(0), ctypes.c_int64(0)
                buf = np.zeros(3 * max(int(n_merges), 1), dtype=np.int64)
                self._chk(self.L.geobpe_run_exchange_log(self._ctx, int(n_merges), ctypes.byref(n), ctypes.byref(first),
                                                         _p(buf), int(n_merges)))
                self._collapsed = bool(self.L.geobpe_collapsed(self._ctx))
                if first.value >= 0 and first.value == len(self.merges):
                    self.merges.extend(tuple(int(x) for x in buf[3 * i:3 * i + 3]) for i in range(n.value))
                else:
                    self._refresh_log()
                if n.value < n_merges:
                    self._done = True
                return int(n.value)
            if self.pipelined and hasattr(self.group, "run_pipelined"):
                done = self.group.run_pipelined(self, int(n_merges))
                self._collapsed = bool(self.L.geobpe_collapsed(self._ctx))
                self._refresh_log()
                if done < n_merges:
                    self._done = True
                return done
            done = 0
            for _ in range(n_merges):
                if self.step(want_merged=False) is None:
                    break
                done += 1
            return done
        n, first = ctypes.c_int64(0), ctypes.c_int64(0)
        buf = np.zeros(3 * max(int(n_merges), 1), dtype=np.int64)
        # (the run's merges come back with it: no further synchronisation for the merge list)
        self._chk(self.L.geobpe_run_log(self._ctx, int(n_merges), ctypes.byref(n), ctypes.byref(first), _p(buf),
                                        int(n_merges)))
        if first.value == len(self.merges):
            self.merges.extend(tuple(int(x) for x in buf[3 * i:3 * i + 3]) for i in range(n.value))
        else:
            self._refresh_log()
        if n.value < n_merges:
            self._done = True
        return int(n.value)

    def _refresh_log(self):
        m = int(self.L.geobpe_merge_log(self._ctx, None, 0))
        if m < 0:
            raise _native.GeoBPEError("merge log unavailable")
        if m > len(self.merges):
            buf = np.zeros(3 * m, dtype=np.int64)
            self.L.geobpe_merge_log(self._ctx, _p(buf), m)
            self.merges = [tuple(int(x) for x in buf[3 * i:3 * i + 3]) for i in range(m)]

    def synchronize(self):
        self._chk(self.L.geobpe_synchronize(self._ctx))

    # ------------------------------------------------------------ introspection
    @property
    def vocab_count(self) -> int:
        return int(self.L.geobpe_vocab_count(self._ctx))

    @property
    def vocab_size(self) -> int:
        return self.vocab_count + 3 * self.B

    @property
    def num_keys(self) -> int:
        return int(self.L.geobpe_num_keys(self._ctx))

    @property
    def num_tokens(self) -> int:
        return int(self.L.geobpe_num_tokens(self._ctx))

    def token_json(self, v: int) -> str:
        m = self.L.geobpe_token_json(self._ctx, v, None, 0)
        if m < 0:
            raise IndexError(v)
        buf = ctypes.create_string_buffer(int(m) + 1)
        self.L.geobpe_token_json(self._ctx, v, buf, m + 1)
        return buf.value.decode()

    def token_content(self, v: int) -> np.ndarray:
        m = self.L.geobpe_token_content(self._ctx, v, None, 0)
        if m < 0:
            raise IndexError(v)
        out = np.empty(m, dtype=np.int32)
        self.L.geobpe_token_content(self._ctx, v, _p(out), m)
        return out

    def merge_keys(self):
        """[(key_json, count)] of every merge so far -- the reference's merge list."""
        if not self.distributed:
            self._refresh_log()
        return [(self.token_json(nid), c) for nid, c, _ in self.merges]

    def key_json(self, d: int) -> str:
        m = self.L.geobpe_key_json(self._ctx, d, None, 0)
        if m < 0:
            raise IndexError(d)
        buf = ctypes.create_string_buffer(int(m) + 1)
        self.L.geobpe_key_json(self._ctx, d, buf, m + 1)
        return buf.value.decode()

    def _keys_and_counts(self):
        U = int(self.L.geobpe_debug_counts(self._ctx, None, None, 0))
        keys = np.zeros(max(U, 1), dtype=np.int32)
        cnt = np.zeros(max(U, 1), dtype=np.int32)
        self.L.geobpe_debug_counts(self._ctx, _p(keys), _p(cnt), U)
        live = keys[:U] >= 0
        return keys[:U][live], cnt[:U][live]

    def key_counts(self) -> dict:
        """{key string: global count} of every key with a positive count."""
        keys, cnt = self._keys_and_counts()
        return {self.key_json(int(d)): int(c) for d, c in zip(keys, cnt) if c > 0}

    def live_key_ids(self) -> np.ndarray:
        """ids (key-table slots) of every key"""
        return self._keys_and_counts()[0].copy()

    def debug_key_less(self, pairs: np.ndarray) -> np.ndarray:
        pairs = np.ascontiguousarray(pairs, dtype=np.int32).reshape(-1, 2)
        out = np.zeros(len(pairs), dtype=np.int32)
        self._chk(self.L.geobpe_debug_key_less(self._ctx, _p(pairs), len(pairs), _p(out)))
        bad = np.flatnonzero(out >= 2)  # 2: the two device comparators disagree
        if len(bad):
            raise _native.GeoBPEError(f"device key order inconsistent on {len(bad)} pairs, first {pairs[bad[0]]} "
                                      f"(code {out[bad[0]]})")
        return out.astype(bool)

    def segmentation(self):
        T = self.L.geobpe_segmentation(self._ctx, None, None, None)
        if T < 0:
            raise _native.GeoBPEError("segmentation failed")
        start = np.empty(T, np.int32)
        ids = np.empty(T, np.int32)
        off = np.empty(self.n_rows + 1, np.int64)
        self.L.geobpe_segmentation(self._ctx, _p(start), _p(ids), _p(off))
        return start, ids, off

    def encode(self):
        T = self.L.geobpe_encode(self._ctx, None, None)
        if T < 0:
            raise _native.GeoBPEError("encode failed")
        ids = np.empty(T, np.int32)
        off = np.empty(self.n_rows + 1, np.int64)
        self.L.geobpe_encode(self._ctx, _p(ids), _p(off))
        return ids, off

    def record_events(self, on: bool = True):
        """Log every merged occurrence from now on (before the first merge): the
        checkpoint's merge tree (geobpe.refpickle)."""
        self._chk(self.L.geobpe_set_record_events(self._ctx, 1 if on else 0))
        self._events_on = bool(on)

    def events(self):
        """(a, b, off): left / right token start slots of the merged occurrences,
        merge t's events in [off[t], off[t+1]), ascending slot within a merge."""
        n = self.L.geobpe_events(self._ctx, None, None, None)
        if n < 0:
            raise _native.GeoBPEError(f"geobpe_events: {self.L.geobpe_last_error(self._ctx).decode()}")
        t = np.empty(n, np.int32)
        a = np.empty(n, np.int32)
        b = np.empty(n, np.int32)
        if n:
            self.L.geobpe_events(self._ctx, _p(t), _p(a), _p(b))
        order = np.lexsort((a, t))
        t, a, b = t[order], a[order], b[order]
        off = np.searchsorted(t, np.arange(len(self.merges) + 1), side="left").astype(np.int64)
        return a, b, off

    def verify_counts(self) -> int:
        n = int(self.L.geobpe_verify_counts(self._ctx))
        if n < 0:
            raise _native.GeoBPEError(_native.lib().geobpe_last_error(self._ctx).decode())
        return n

    # ------------------------------------------------------------ profiling
    def set_profiling(self, on: bool = True, only: str = "", stride: int = 1):
        """HIP-event timing of the named kernels ("" = all), every ``stride``-th launch."""
        self._chk(self.L.geobpe_set_profiling_filter(self._ctx, only.encode()))
        self._chk(self.L.geobpe_set_profiling(self._ctx, max(1, int(stride)) if on else 0))

    def set_hold(self, us: int = 0):
        """A spin kernel of ``us`` microseconds before each batch of run() (event timing)."""
        self._chk(self.L.geobpe_set_hold(self._ctx, int(us)))

    def set_work_counters(self, on: bool = True):
        """k_commit's work counters (state() keys commit_*) on or off."""
        self._chk(self.L.geobpe_set_work_counters(self._ctx, 1 if on else 0))

    def state(self) -> dict:
        """Loop state (hot list, threshold, posting index) after a synchronisation."""
        v = np.zeros(13, dtype=np.int64)
        n = self.L.geobpe_debug_state(self._ctx, _p(v), 13)
        if n < 0:
            self._chk(int(n))
        keys = ("hot_list", "theta", "ncand", "maxc", "nskip", "cl_valid", "iter", "K", "post_valid", "pool_used",
                "commit_key_records", "commit_decrement_records", "commit_keys")
        return {k: int(x) for k, x in zip(keys, v)}

    def marker(self, tag: int = 0):
        """Enqueue the empty k_window_mark kernel (brackets a profiled window)."""
        self._chk(self.L.geobpe_marker(self._ctx, int(tag)))

    def kernel_ms(self, name: str):
        n = ctypes.c_int64(0)
        ms = self.L.geobpe_kernel_ms(self._ctx, name.encode(), ctypes.byref(n))
        return float(ms), int(n.value)
