"""The multi-rank exchange layer on CPU: world_size 2 over gloo (127.0.0.1).

Covers what the N>1 path does on the host between device calls: the
threshold / first-appearance all-reduces and the variable-size all-gather of
40-byte delta records.  The device side of the protocol is covered on the GPU
by tests/test_gpu_parity.py (VirtualCluster, several shards on one device)."""
import os
import socket

import numpy as np
import pytest

REC = 40


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    import ctypes
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(os.path.dirname(here), "pt-bpe_amd"))
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from geobpe.dist import TorchGroup
        R_local = 100 + 50 * rank
        g = TorchGroup(R_local)
        assert g.residue_base == (0 if rank == 0 else 100)
        assert g.total_residues == 250
        mm = np.array([rank + 0.5, rank + 2.0] * 6)
        cnt = np.arange(6, dtype=np.int64) + rank
        mm2, cnt2, nrows = g.reduce_ranges(mm, cnt, 10 + rank)
        assert mm2[0] == 0.5 and mm2[1] == 3.0
        assert list(cnt2) == [2 * i + 1 for i in range(6)] and nrows == 21
        first = np.array([5, 7, np.iinfo(np.int64).max], dtype=np.int64) - rank
        assert list(g.reduce_first(first)[:2]) == [4, 6]
        # export buffer -> variable-length all-gather of records
        cap, ptr = g.export_buffer(None)
        n = 3 + 2 * rank
        payload = np.arange(n * REC, dtype=np.uint8) % 251 + rank
        ctypes.memmove(ptr.value, payload.ctypes.data, n * REC)
        d, total = g.all_gather_deltas(None, n)
        got = np.ctypeslib.as_array((ctypes.c_uint8 * (total * REC)).from_address(d.value)).copy()
        exp = np.concatenate([np.arange((3 + 2 * r) * REC, dtype=np.uint8) % 251 + r for r in range(world)])
        assert total == 8 and np.array_equal(got, exp)
        q.put((rank, "ok"))
    except Exception as e:  # pragma: no cover
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


def test_torchgroup_gloo_world2():
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=240) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    assert res == {0: "ok", 1: "ok"}


def _engine_worker(rank, world, port, q, mode="pipelined"):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(os.path.dirname(here), "pt-bpe_amd"))
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from geobpe import synth
        from geobpe.dist import TorchGroup, shard_rows, slice_corpus
        from geobpe.engine import GeoBPEEngine
        corpus = synth.make_corpus(synth.make_lengths(2000, 20, 300, seed=91), seed=91, repeat_frac=0.05)
        lo, hi = shard_rows(corpus["row_off"], world)[rank]
        mid = None
        # the sharded exchange to the end, or (modes "collapse*", "skewed", "mixed-collapse") the
        # collapse at the middle-regime switch: every rank goes on with the whole corpus
        collapse = mode.startswith("collapse") or mode in ("skewed", "mixed-collapse")
        if mode.startswith("skewed"):
            # rank 0 holds 5 % of the rows: its own merged counts sit far below the others', so
            # a switch to the middle regime decided per rank would part the ranks' collectives
            # (ADVICE r3); the switch must follow the replicated winner count (mid = 1500 puts
            # it inside the run)
            cuts = [0, 100] + [100 + (1900 * (r + 1)) // (world - 1) for r in range(world - 1)]
            lo, hi = cuts[rank], cuts[rank + 1]
            mid = 1500
        shard = slice_corpus(corpus, lo, hi)
        g = TorchGroup(int(shard["row_off"][-1]), device=0)
        if mode.endswith("small-slots"):  # most merges overflow the fixed slots: the stall / resolve path
            g.pipe_cap = 16
        if mode.startswith("allgather"):  # the all-gather of fixed slots instead of the peer exchange
            g.peer = False
        if mode == "host-loop":  # the Python-driven loop (geobpe.dist) instead of geobpe_run_exchange
            g.engine_exchange = False
        e = GeoBPEEngine(shard, 5, device=0, group=g, mid=mid, collapse=collapse).initialize()
        e.pipelined = mode != "stepwise"
        e.bin()
        done = e.run(70)
        if mode.startswith("mixed"):  # pipelined -> host-synchronised step() -> pipelined: the parity hand-offs
            for _ in range(20):
                done += e.step(want_merged=False) is not None
            done += e.run(60)
        else:
            done += e.run(80)  # a second pipelined run continues the device parity
        s, ids, off = e.segmentation()
        if mode not in ("stepwise", "host-loop"):  # (geobpe_run_exchange ran: which exchange it took)
            assert e.L.geobpe_comm_peer_active(e._ctx) == (0 if mode.startswith("allgather") else 1)
        if mode.startswith("skewed"):
            assert e.merges[0][1] > mid >= e.merges[-1][1], "the run does not cross the middle-regime threshold"
        assert e.collapsed == collapse, "collapse expected" if collapse else "no collapse expected"
        if collapse:  # the whole corpus on every rank: its counts are the global ones
            assert e.verify_counts() == 0, "counts after the collapse differ from a full recount"
            assert len(off) == hi - lo + 1 and e.encode()[1].shape == off.shape  # (this rank's rows only)
        q.put((rank, done, e.merge_keys(), ids.tolist()))
    except Exception as ex:  # pragma: no cover
        q.put((rank, -1, repr(ex), None))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("world, mode", [(2, "pipelined"), (3, "pipelined"), (2, "small-slots"), (2, "stepwise"),
                                         (3, "mixed"), (4, "small-slots"), (2, "host-loop"), (2, "allgather"),
                                         (3, "allgather-small-slots"),
                                         (2, "skewed-nocollapse"), (3, "skewed-nocollapse"), (2, "skewed"),
                                         (3, "skewed"), (2, "collapse"), (4, "collapse"), (2, "mixed-collapse")])
def test_multirank_engine_on_one_gpu_matches_single(world, mode, oracle_lib):
    """The full N>1 path (TorchGroup exchange, one process per rank) with gloo on
    one device: the engine's pipelined loop (geobpe_run_exchange: the peer exchange -- every
    rank's receive area IPC-mapped into the others, records stored by the merge kernels, the
    stream waiting on the peers' headers -- or, "allgather*", the group's host collective over
    fixed slots; stall + full re-exchange of an overflowing merge), the same with tiny slots,
    the Python-driven loop, and the host-synchronised per-merge
    exchange; skewed shards whose own merged counts cross the middle-regime threshold far
    apart (the switch follows the replicated count); the collapse at that switch (every
    rank gathers the whole corpus and goes on alone) early, mid-run and before host steps.
    Merge list and segmentation equal the oracle's."""
    import multiprocessing as mp
    from geobpe import synth
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_engine_worker, args=(r, world, port, q, mode)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=300) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    assert all(r[1] == 150 for r in res), res[0][2] if res[0][1] < 0 else None
    corpus = synth.make_corpus(synth.make_lengths(2000, 20, 300, seed=91), seed=91, repeat_frac=0.05)
    o = oracle_lib.OracleBPE(corpus, 5).initialize()
    o.bin()
    for _ in range(150):
        o.step()
    assert all(r[2] == o.merges for r in res)
    _, ids, _ = o.segmentation()
    assert sum((r[3] for r in res), []) == ids.tolist()


def test_rank_plan_replicates_below_the_measured_crossover(monkeypatch):
    """bench.py's choice per world size (geobpe.dist.rank_plan): replicas below SHARD_MIN_RANKS,
    where one rank's share with the exchange measured slower than the whole corpus alone."""
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(os.path.dirname(here), "pt-bpe_amd"))
    from geobpe.dist import SHARD_MIN_RANKS, rank_plan

    monkeypatch.delenv("GEOBPE_RANK_PLAN", raising=False)
    assert SHARD_MIN_RANKS == 4
    assert [rank_plan(w) for w in (1, 2, 3, 4, 8)] == ["replicate", "replicate", "replicate", "shard", "shard"]
    monkeypatch.setenv("GEOBPE_RANK_PLAN", "shard")
    assert rank_plan(2) == "shard" and rank_plan(1) == "replicate"
    monkeypatch.setenv("GEOBPE_RANK_PLAN", "rows")
    with pytest.raises(ValueError):
        rank_plan(2)
