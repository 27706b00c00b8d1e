"""Row-sharded multi-GPU GeoBPE.

One process per GPU, ``torch.distributed`` over RCCL (backend "nccl") or gloo.
The corpus is split into contiguous blocks of chains balanced by residue count
(`shard_rows`); global row order is kept, so first-appearance labels and the
merge list are identical to the single-GPU run.

Per iteration every rank selects the same winner from its replicated copy of the
global pair counts, applies it to its own chains, and the ranks exchange their
count deltas: one all-gather of the record counts and one all-gather of the
40-byte delta records (hash, length, representative, delta) of every key whose
local count changed.  Keys are matched by content hash, so ranks never need a
shared dense numbering.

`VirtualCluster` runs the same protocol with several shards in ONE process on
one device (each shard its own context); the GPU parity tests use it to check
the sharded path against the oracle without needing several GPUs.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _native
from .engine import GeoBPEEngine, ANGLE_TYPES

REC = _native.DELTA_RECORD_BYTES

# The fewest ranks at which row sharding beats every rank running the whole corpus alone.  One
# rank's share with the peer exchange (loopback), against the whole corpus on the same GPU, on
# the driver window (profiles/r6_final/suite/fx_w{2,4,8}.json): 1/2 0.81 x, 1/4 1.08 x,
# 1/8 1.28 x.  Below it the ranks are replicas: each holds the whole corpus and runs the one-rank
# loop, so the job runs at the one-GPU rate instead of 0.8 x of it.
SHARD_MIN_RANKS = 4


def rank_plan(world: int) -> str:
    """'shard' (rows split over the ranks, the peer exchange) or 'replicate' (every rank the
    whole corpus, no exchange) for a run of `world` ranks.  GEOBPE_RANK_PLAN=shard|replicate
    overrides the measured choice (rehearsals, tests)."""
    import os

    forced = os.environ.get("GEOBPE_RANK_PLAN")
    if forced is not None:
        if forced not in ("shard", "replicate"):
            raise ValueError(f"GEOBPE_RANK_PLAN must be 'shard' or 'replicate', not {forced!r}")
        return forced if world > 1 else "replicate"
    return "shard" if world >= SHARD_MIN_RANKS else "replicate"


def shard_rows(row_off: np.ndarray, world: int) -> list:
    """Contiguous chain blocks [(row_lo, row_hi)] with ~equal residue counts."""
    row_off = np.asarray(row_off, dtype=np.int64)
    n = len(row_off) - 1
    R = int(row_off[-1])
    bounds = [0]
    for r in range(1, world):
        target = R * r / world
        b = int(np.searchsorted(row_off, target, side="left"))
        b = min(max(b, bounds[-1]), n)
        bounds.append(b)
    bounds.append(n)
    return [(bounds[i], bounds[i + 1]) for i in range(world)]


def slice_corpus(corpus: dict, lo: int, hi: int) -> dict:
    ro = np.asarray(corpus["row_off"], dtype=np.int64)
    a, b = int(ro[lo]), int(ro[hi])
    out = {k: v[a:b] for k, v in corpus.items() if k != "row_off"}
    out["row_off"] = ro[lo:hi + 1] - a
    return out


class TorchGroup:
    """Exchange over torch.distributed (nccl = RCCL on ROCm, or gloo)."""

    def __init__(self, R_local: int, device: int = 0, pg=None):
        import torch
        import torch.distributed as dist
        self.torch, self.dist, self.pg = torch, dist, pg
        self.rank = dist.get_rank(pg)
        self.world_size = dist.get_world_size(pg)
        self.backend = dist.get_backend(pg)
        self.on_gpu = self.backend == "nccl"
        self.dev = torch.device("cuda", device) if torch.cuda.is_available() else torch.device("cpu")
        self.comm_dev = self.dev if self.on_gpu else torch.device("cpu")
        sizes = self._gather_i64(R_local)
        self.residue_base = int(sum(sizes[: self.rank]))
        self.total_residues = int(sum(sizes))
        self.R_local = R_local
        self._buf = None

    def _gather_i64(self, x: int) -> list:
        t = self.torch.tensor([int(x)], dtype=self.torch.int64, device=self.comm_dev)
        out = [self.torch.zeros_like(t) for _ in range(self.world_size)]
        self.dist.all_gather(out, t, group=self.pg)
        return [int(o.item()) for o in out]

    def reduce_ranges(self, mm: np.ndarray, cnt: np.ndarray, n_rows: int):
        T = self.torch
        mins = T.tensor(mm[0::2].copy(), dtype=T.float64, device=self.comm_dev)
        maxs = T.tensor(mm[1::2].copy(), dtype=T.float64, device=self.comm_dev)
        c = T.tensor(np.append(cnt, n_rows), dtype=T.int64, device=self.comm_dev)
        self.dist.all_reduce(mins, op=self.dist.ReduceOp.MIN, group=self.pg)
        self.dist.all_reduce(maxs, op=self.dist.ReduceOp.MAX, group=self.pg)
        self.dist.all_reduce(c, op=self.dist.ReduceOp.SUM, group=self.pg)
        out = np.empty(12)
        out[0::2] = mins.cpu().numpy()
        out[1::2] = maxs.cpu().numpy()
        cc = c.cpu().numpy()
        return out, cc[:6], int(cc[6])

    def reduce_first(self, first: np.ndarray) -> np.ndarray:
        t = self.torch.tensor(first, dtype=self.torch.int64, device=self.comm_dev)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MIN, group=self.pg)
        return t.cpu().numpy()

    def export_buffer(self, engine):
        if self._buf is None:
            cap = 3 * self.R_local + 65536  # keys touched by one merge: <= 5 per occurrence, <= R/2 occurrences
            self._buf = self.torch.empty(cap * REC, dtype=self.torch.uint8, device=self.dev)
            self._cap = cap
        return self._cap, ctypes.c_void_p(self._buf.data_ptr())

    def all_gather_deltas(self, engine, n: int):
        T = self.torch
        counts = self._gather_i64(n)
        m = max(counts)
        if m == 0:
            return ctypes.c_void_p(self._buf.data_ptr()), 0
        src = self._buf[: m * REC]
        if not self.on_gpu:
            src = src.cpu()
        out = T.empty(self.world_size * m * REC, dtype=T.uint8, device=src.device)
        self.dist.all_gather_into_tensor(out, src, group=self.pg)
        out = out.view(self.world_size, m * REC)
        parts = [out[r, : counts[r] * REC] for r in range(self.world_size)]
        flat = T.cat(parts).to(self.dev)
        self._keep = flat
        # the engine runs on its own HIP stream: the records must be complete on
        # torch's stream before the import kernels read them
        if self.dev.type == "cuda":
            T.cuda.current_stream(self.dev).synchronize()
        return ctypes.c_void_p(flat.data_ptr()), int(sum(counts))


    # ---------------------------------------------------------------- pipelined exchange
    PIPE_CAP_MIN, PIPE_CAP_MAX = 1024, 65536  # records per rank slot (40 B each)
    PIPE_AHEAD = 64      # iterations enqueued between polls (doubling from 1 after a stall)
    engine_exchange = True  # the loop and its collectives in the engine (geobpe_run_exchange)

    def _host_allgather(self, user, hsend, hrecv, nbytes):
        """geobpe_allgather_fn over this group (gloo): host bytes of every rank, rank-major."""
        try:
            T = self.torch
            src = np.ctypeslib.as_array((ctypes.c_uint8 * int(nbytes)).from_address(hsend)).copy()
            out = T.empty(self.world_size * int(nbytes), dtype=T.uint8)
            self.dist.all_gather_into_tensor(out, T.from_numpy(src), group=self.pg)
            ctypes.memmove(hrecv, out.numpy().ctypes.data, self.world_size * int(nbytes))
            return 0
        except Exception:  # pragma: no cover - reported by the engine as a failed exchange
            return 1

    def attach(self, engine):
        """The engine's own exchange: an RCCL communicator (backend nccl: rank 0's id
        broadcast over this group) or this group's host collective (gloo)."""
        if getattr(engine, "_x_attached", False):
            return
        L, T = engine.L, self.torch
        if self.backend == "nccl":
            path = _native.rccl_path()
            pb = path.encode() if path else None
            uid = np.zeros(128, dtype=np.uint8)
            if self.rank == 0:
                rc = L.geobpe_comm_unique_id(pb, uid.ctypes.data_as(ctypes.c_void_p))
                if rc:
                    raise _native.GeoBPEError(f"geobpe_comm_unique_id: {L.geobpe_comm_error().decode()}")
            t = T.from_numpy(uid).to(self.comm_dev)
            self.dist.broadcast(t, src=0, group=self.pg)
            uid = t.cpu().numpy()
            engine._chk(L.geobpe_comm_init_rccl(engine._ctx, pb, uid.ctypes.data_as(ctypes.c_void_p),
                                                self.world_size, self.rank))
        else:
            self._cb = _native.ALLGATHER_FN(self._host_allgather)  # (kept alive with the group)
            engine._chk(L.geobpe_comm_set_callback(engine._ctx, ctypes.cast(self._cb, ctypes.c_void_p), None,
                                                   self.world_size, self.rank))
        fixed = getattr(self, "pipe_cap", None)
        if fixed:
            engine._chk(L.geobpe_comm_set_slot(engine._ctx, int(fixed)))
        peer = getattr(self, "peer", None)  # (None: the engine's default, the peer exchange up to 8 ranks)
        if peer is not None:
            engine._chk(L.geobpe_comm_peer(engine._ctx, 1 if peer else 0))
        engine._x_attached = True

    def run_pipelined(self, engine, n_merges: int) -> int:
        if self.engine_exchange:
            self.attach(engine)
            n = ctypes.c_int64(0)
            engine._chk(engine.L.geobpe_run_exchange(engine._ctx, int(n_merges), ctypes.byref(n)))
            return int(n.value)
        return self._run_pipelined_host(engine, n_merges)

    def _run_pipelined_host(self, engine, n_merges: int) -> int:
        """``n_merges`` merges with no host wait per merge (include/geobpe.h,
        geobpe_pipeline_*): per iteration the engine enqueues select / mark / apply
        and its export into a fixed slot, one all-gather of the slots follows on the
        engine's stream, then the import.  The host polls every few iterations; a
        merge whose records overflowed a slot stalls the device until it is
        re-exchanged in full (`_resolve`).  Slots are sized per poll window from the
        largest count of the last import (2x, a power of two, clamped): the merges'
        counts shrink as training goes on, and so do the collectives.  Every rank
        sees the same poll results, so every rank issues the same collectives."""
        T, L, ctx = self.torch, engine.L, engine._ctx
        W = self.world_size
        fixed = getattr(self, "pipe_cap", None)  # tests: a fixed slot size
        if getattr(self, "_pbuf", None) is None:
            self._pcap = 3 * self.R_local + 65536
            self._pbuf = T.zeros((1 + self._pcap) * REC, dtype=T.uint8, device=self.dev)
            top = int(fixed) if fixed else self.PIPE_CAP_MAX
            self._gath = T.empty(W * (1 + top) * REC, dtype=T.uint8, device=self.comm_dev)
        pbuf = ctypes.c_void_p(self._pbuf.data_ptr())
        out = (ctypes.c_int64 * 4)()
        engine._chk(L.geobpe_pipeline_begin(ctx))
        ok = False
        try:
            engine._chk(L.geobpe_pipeline_poll(ctx, out))
            # the poll window and the slot size carry over from the last call (a run of
            # merges is often split into several calls: warm-up, timed window)
            it0, done, ahead = int(out[1]), 0, getattr(self, "_ahead", 1)
            capf = int(fixed) if fixed else getattr(self, "_capf", self.PIPE_CAP_MIN)
            with T.cuda.stream(engine.torch_stream):
                while done < n_merges:
                    slot = (1 + capf) * REC
                    gath = self._gath[: W * slot]
                    for _ in range(min(ahead, n_merges - done)):  # an iteration merges at most once
                        engine._chk(L.geobpe_pipeline_iter(ctx, pbuf, self._pcap))
                        src = self._pbuf[:slot]
                        if self.on_gpu:
                            self.dist.all_gather_into_tensor(gath, src, group=self.pg)
                            g = gath
                        else:  # gloo: through host copies
                            self.dist.all_gather_into_tensor(gath, src.cpu(), group=self.pg)
                            g = gath.to(self.dev)
                            self._keep = g
                        engine._chk(L.geobpe_pipeline_import(ctx, ctypes.c_void_p(g.data_ptr()), W, capf))
                    engine._chk(L.geobpe_pipeline_poll(ctx, out))
                    stalled, it, fin, smax = (int(x) for x in out)
                    if stalled:
                        self._resolve(engine)
                        ahead = 1
                    else:
                        ahead = min(2 * ahead, self.PIPE_AHEAD)
                    if not fixed:
                        capf = min(self.PIPE_CAP_MAX, max(self.PIPE_CAP_MIN, 1 << (2 * max(smax, 1) - 1).bit_length()))
                    done = it - it0
                    self._ahead, self._capf = ahead, capf
                    if fin:
                        break
            ok = True
        finally:
            rc = L.geobpe_pipeline_end(ctx)
            if ok:  # (an error in flight is the one to report)
                engine._chk(rc)
        return done

    def _resolve(self, engine):
        """The stalled merge's full records: counts from the slot headers, then the
        records (sized by the largest count), imported on every rank."""
        T = self.torch
        cnt = self._pbuf[:8].view(T.int64)
        src = cnt if self.on_gpu else cnt.cpu()
        allc = T.empty(self.world_size, dtype=T.int64, device=src.device)
        self.dist.all_gather_into_tensor(allc, src, group=self.pg)
        counts = [int(x) for x in allc.cpu().tolist()]
        m = max(counts)
        if m > self._pcap:
            raise _native.GeoBPEError(f"delta export needs {m} records (cap {self._pcap})")
        src = self._pbuf[REC: REC + m * REC]
        if not self.on_gpu:
            src = src.cpu()
        out = T.empty(self.world_size * m * REC, dtype=T.uint8, device=src.device)
        self.dist.all_gather_into_tensor(out, src, group=self.pg)
        out = out.view(self.world_size, m * REC)
        flat = T.cat([out[r, : counts[r] * REC] for r in range(self.world_size)]).to(self.dev)
        engine._chk(engine.L.geobpe_pipeline_resolve(engine._ctx, ctypes.c_void_p(flat.data_ptr()),
                                                      int(sum(counts))))

    def exchange_async(self, engine):
        """One merge's exchange with two host waits in all: the export count is
        written on the device and all-gathered, the host reads the counts (the
        only sync), then the records are all-gathered and imported stream-ordered
        (ProcessGroupNCCL orders the collectives after / before the engine's
        kernels on the current stream; gloo goes through host copies)."""
        T = self.torch
        with T.cuda.stream(engine.torch_stream):
            self._exchange_on_stream(engine)

    def _exchange_on_stream(self, engine):
        T = self.torch
        cap, ptr = self.export_buffer(engine)
        if getattr(self, "_cnt", None) is None:
            self._cnt = T.zeros(1, dtype=T.int64, device=self.dev)
        engine._chk(engine.L.geobpe_delta_export_async(engine._ctx, ptr, cap, ctypes.c_void_p(self._cnt.data_ptr())))
        src = self._cnt if self.on_gpu else self._cnt.cpu()
        allc = T.empty(self.world_size, dtype=T.int64, device=src.device)
        self.dist.all_gather_into_tensor(allc, src, group=self.pg)
        counts = [int(x) for x in allc.cpu().tolist()]  # the merge's one host wait on the exchange
        if max(counts) > cap:
            raise _native.GeoBPEError(f"delta export needs {max(counts)} records (cap {cap})")
        m = max(counts)
        if m == 0:
            return
        src = self._buf[: m * REC]
        if not self.on_gpu:
            src = src.cpu()
        out = T.empty(self.world_size * m * REC, dtype=T.uint8, device=src.device)
        self.dist.all_gather_into_tensor(out, src, group=self.pg)
        out = out.view(self.world_size, m * REC)
        flat = T.cat([out[r, : counts[r] * REC] for r in range(self.world_size)]).to(self.dev)
        self._keep = flat
        engine._chk(engine.L.geobpe_delta_import_async(engine._ctx, ctypes.c_void_p(flat.data_ptr()),
                                                       int(sum(counts))))


class _VirtualGroup:
    """Rank view inside a VirtualCluster (only the attributes the engine reads)."""

    def __init__(self, cluster, rank):
        self.cluster, self.rank = cluster, rank
        self.world_size = cluster.world


class VirtualCluster:
    """k row shards in one process on one device, run in lockstep with the exact
    multi-rank protocol (replicated counts, delta exchange)."""

    def __init__(self, corpus: dict, bins: int, world: int, device: int = 0, max_vocab: int = 1 << 20,
                 cover: bool = False):
        import torch
        self.torch = torch
        self.world = world
        self.bounds = shard_rows(corpus["row_off"], world)
        self.shards = [slice_corpus(corpus, lo, hi) for lo, hi in self.bounds]
        self.engines = [GeoBPEEngine(s, bins, device=device, max_vocab=max_vocab) for s in self.shards]
        self.R = [int(s["row_off"][-1]) for s in self.shards]
        self.base = [int(sum(self.R[:r])) for r in range(world)]
        self.B = int(bins)
        self.cover = bool(cover)
        self.dev = torch.device("cuda", device)
        self.merges = []

    def initialize(self):
        L = _native.lib()
        from .engine import init_bond_angle, histogram_edges, TWO_PI, _p
        mms, cnts = [], []
        for e in self.engines:
            arr = (ctypes.c_void_p * 9)(*[c.ctypes.data for c in e._cols])
            e._chk(L.geobpe_load_angles(e._ctx, e.n_rows, _p(e.row_off), arr))
            mm = np.zeros(12)
            cnt = np.zeros(6, dtype=np.int64)
            e._chk(L.geobpe_angle_range(e._ctx, _p(mm), _p(cnt)))
            mms.append(mm)
            cnts.append(cnt)
        mm = np.empty(12)
        mm[0::2] = np.min([m[0::2] for m in mms], axis=0)
        mm[1::2] = np.max([m[1::2] for m in mms], axis=0)
        cnt = np.sum(cnts, axis=0)
        n_rows = sum(e.n_rows for e in self.engines)
        w0 = (init_bond_angle() + TWO_PI) % TWO_PI
        edges = np.zeros((6, self.B + 1))
        thr = {}
        for t, key in enumerate(ANGLE_TYPES):
            mn, mx, c = float(mm[2 * t]), float(mm[2 * t + 1]), int(cnt[t])
            if key == "tau" and n_rows > 0:
                mn, mx, c = (min(mn, w0), max(mx, w0), c + n_rows) if c > 0 else (w0, w0, n_rows)
            e_ = histogram_edges(mn, mx, c, self.B, self.cover)
            edges[t] = e_
            thr[key] = [(float(s), float(f)) for s, f in zip(e_[:-1], e_[1:])]
        self.thresholds = thr
        S = self.B ** 3 + self.B
        first = np.full(S, np.iinfo(np.int64).max, dtype=np.int64)
        for r, e in enumerate(self.engines):
            e._chk(L.geobpe_quantize(e._ctx, self.B, _p(edges), init_bond_angle()))
            f = np.zeros(S, dtype=np.int64)
            e._chk(L.geobpe_symbol_first(e._ctx, self.base[r], _p(f)))
            first = np.minimum(first, f)
        present = np.nonzero(first != np.iinfo(np.int64).max)[0]
        order = present[np.argsort(first[present], kind="stable")]
        lab = np.full(S, -1, dtype=np.int32)
        lab[order] = np.arange(len(order), dtype=np.int32)
        self.K0 = len(order)
        for e in self.engines:
            e._chk(L.geobpe_init_tokens(e._ctx, _p(lab), self.K0))
            e.K0 = self.K0
            e._initialized = True
        return self

    def _exchange(self):
        L = _native.lib()
        T = self.torch
        parts = []
        for e, R in zip(self.engines, self.R):
            cap = R + 65536
            buf = T.empty(cap * REC, dtype=T.uint8, device=self.dev)
            n = ctypes.c_int64(0)
            e._chk(L.geobpe_delta_export(e._ctx, ctypes.c_void_p(buf.data_ptr()), cap, ctypes.byref(n)))
            parts.append(buf[: n.value * REC])
        flat = T.cat(parts)
        total = flat.numel() // REC
        T.cuda.current_stream(self.dev).synchronize()  # engines run on their own streams
        for e in self.engines:
            e._chk(L.geobpe_delta_import(e._ctx, ctypes.c_void_p(flat.data_ptr()), total))

    def bin(self):
        L = _native.lib()
        total = sum(self.R)
        for e in self.engines:
            e._chk(L.geobpe_set_distributed(e._ctx, 1))
            e._chk(L.geobpe_set_global_residues(e._ctx, total))
            e._chk(L.geobpe_bin(e._ctx))
        self._exchange()

    def step(self):
        L = _native.lib()
        sel = []
        for e in self.engines:
            nid, cnt = ctypes.c_int32(0), ctypes.c_int32(0)
            e._chk(L.geobpe_step_select(e._ctx, ctypes.byref(nid), ctypes.byref(cnt)))
            sel.append((nid.value, cnt.value))
        if len(set(sel)) != 1:
            raise _native.GeoBPEError(f"ranks disagree on the winner: {sel}")
        if sel[0][0] < 0:
            return None
        nm_total = 0
        for e in self.engines:
            nm = ctypes.c_int64(0)
            e._chk(L.geobpe_step_apply(e._ctx, ctypes.byref(nm)))
            nm_total += nm.value
        self._exchange()
        rec = (sel[0][0], sel[0][1], nm_total)
        self.merges.append(rec)
        for e in self.engines:
            e.merges.append(rec)
        return rec

    def merge_keys(self):
        e = self.engines[0]
        return [(e.token_json(nid), c) for nid, c, _ in self.merges]

    def segmentation(self):
        parts = [e.segmentation() for e in self.engines]
        start = np.concatenate([p[0] for p in parts])
        ids = np.concatenate([p[1] for p in parts])
        offs = [0]
        for p in parts:
            offs.extend((p[2][1:] + offs[-1]).tolist())
        return start, ids, np.array(offs, dtype=np.int64)

    def encode(self):
        parts = [e.encode() for e in self.engines]
        ids = np.concatenate([p[0] for p in parts])
        offs = [0]
        for p in parts:
            offs.extend((p[1][1:] + offs[-1]).tolist())
        return ids, np.array(offs, dtype=np.int64)

    def close(self):
        for e in self.engines:
            e.close()
