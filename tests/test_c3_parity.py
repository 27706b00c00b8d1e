"""The north_star target: bit-exact parity on the 10^5-sequence corpus.

BASELINE configs[2] (C3): 100 000 synthetic chains, lengths U{40..560} (~30 M
residues), seed 0, bins {1: 5}, 1000 merges -- the HIP loop (device-resident
``run()``) against the CPU oracle on the same corpus: merge list (key string and
count), segmentation and encoded ids.  configs[4] in its bins {1: 5} form (5000
merges on the same corpus) and configs[3] (the corpus row-sharded
over 8 ranks) are checked against the same oracle run.  Reference semantics:
foldingdiff/bpe.py:1431-1474 (bin), :1792-2166 (step), tokenizer.py:379-392 and
bpe.py:918-956 (encode)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

C3_MERGES = 1000
C5_MERGES = 5000


@pytest.fixture(scope="module")
def c3(oracle_lib):
    from geobpe import synth
    lengths = synth.make_lengths(100_000, 40, 560, seed=0)
    corpus = synth.make_corpus(lengths, seed=0)
    o = oracle_lib.OracleBPE(corpus, 5).initialize()
    o.bin()
    snap = {}
    for target in (C3_MERGES, C5_MERGES):
        while len(o.merges) < target:
            assert o.step() is not None
        snap[target] = dict(merges=list(o.merges), seg=o.segmentation(), enc=o.encode(),
                            thresholds=o.thresholds)
    del o
    return corpus, snap


def _check(run, want):
    assert run.merge_keys() == want["merges"]
    for x, y in zip(run.segmentation(), want["seg"]):
        assert np.array_equal(x, y)
    for x, y in zip(run.encode(), want["enc"]):
        assert np.array_equal(x, y)


@pytest.mark.timeout(600)
def test_c3_1000_merges_match_oracle(c3):
    from geobpe.engine import GeoBPEEngine
    corpus, snap = c3
    eng = GeoBPEEngine(corpus, 5, device=0).initialize()
    assert eng.thresholds == snap[C3_MERGES]["thresholds"]
    eng.bin()
    assert eng.run(C3_MERGES) == C3_MERGES
    _check(eng, snap[C3_MERGES])
    assert eng.verify_counts() == 0
    # configs[4] (bins {1: 5} form): the same loop on to 5000 merges
    assert eng.run(C5_MERGES - C3_MERGES) == C5_MERGES - C3_MERGES
    _check(eng, snap[C5_MERGES])
    assert eng.verify_counts() == 0
    eng.close()


def _c4_rank(rank, world, port, q):
    """One rank of the multi-rank path bench.py runs at N > 1 (TorchGroup + engine.run,
    the pipelined exchange), over gloo with every rank on GPU 0."""
    import os
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from geobpe import synth
        from geobpe.dist import TorchGroup, shard_rows, slice_corpus
        from geobpe.engine import GeoBPEEngine
        corpus = synth.make_corpus(synth.make_lengths(100_000, 40, 560, seed=0), seed=0)
        lo, hi = shard_rows(corpus["row_off"], world)[rank]
        shard = slice_corpus(corpus, lo, hi)
        del corpus
        g = TorchGroup(int(shard["row_off"][-1]), device=0)
        e = GeoBPEEngine(shard, 5, device=0, group=g, max_vocab=1 << 20).initialize()
        e.bin()
        out = {}
        done = e.run(10) + e.run(C3_MERGES - 10)  # warm-up then the rest, as bench.py splits it
        out[C3_MERGES] = (done, e.merge_keys() if rank == 0 else None, _digest(*e.segmentation(), *e.encode()))
        done += e.run(C5_MERGES - C3_MERGES)
        out[C5_MERGES] = (done, e.merge_keys() if rank == 0 else None, _digest(*e.segmentation(), *e.encode()))
        q.put((rank, out))
    except Exception as ex:  # pragma: no cover
        import traceback
        q.put((rank, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


def _digest(start, ids, soff, enc, eoff):
    """sha256 of a shard's segmentation (token starts, ids, row offsets) and encoding"""
    import hashlib
    h = hashlib.sha256()
    for a, dt in ((start, np.int32), (ids, np.int32), (soff, np.int64), (enc, np.int32), (eoff, np.int64)):
        h.update(np.ascontiguousarray(a, dtype=dt).tobytes())
    return h.hexdigest()


def _rows_digest(want, lo, hi):
    """the digest of rows [lo, hi) of a whole-corpus (oracle) segmentation / encoding"""
    start, ids, soff = want["seg"]
    enc, eoff = want["enc"]
    a, b = int(soff[lo]), int(soff[hi])
    c, d = int(eoff[lo]), int(eoff[hi])
    return _digest(start[a:b], ids[a:b], np.asarray(soff[lo:hi + 1]) - a, enc[c:d], np.asarray(eoff[lo:hi + 1]) - c)


@pytest.mark.timeout(1200)
def test_c4_world8_pipelined_ranks_match_oracle(c3):
    """configs[3] / configs[4] at N = 8 through the path bench.py takes at N > 1: 8 rank
    processes (TorchGroup over gloo, all on GPU 0), the pipelined exchange of engine.run;
    1000 merges, then on to 5000, each bit-exact with the 1-rank oracle (merge list,
    segmentation, encoded ids)."""
    import multiprocessing as mp
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    corpus, snap = c3
    world = 8
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_c4_rank, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=1100) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    bad = {r: v for r, v in res.items() if isinstance(v, str)}
    assert not bad, next(iter(bad.values()))
    from geobpe.dist import shard_rows
    bounds = shard_rows(corpus["row_off"], world)
    for target in (C3_MERGES, C5_MERGES):
        want = snap[target]
        assert all(res[r][target][0] == target for r in range(world))
        assert res[0][target][1] == want["merges"]
        for r, (lo, hi) in enumerate(bounds):
            assert res[r][target][2] == _rows_digest(want, lo, hi), f"rank {r} (rows {lo}..{hi}) at {target} merges"


@pytest.mark.timeout(900)
def test_c4_world8_matches_oracle(c3):
    """configs[3]: the C3 corpus row-sharded over 8 ranks (8 engines on one GPU,
    per-merge delta exchange), 1000 merges, bit-exact with the 1-rank oracle."""
    from geobpe.dist import VirtualCluster
    corpus, snap = c3
    vc = VirtualCluster(corpus, 5, world=8).initialize()
    assert vc.thresholds == snap[C3_MERGES]["thresholds"]
    vc.bin()
    for _ in range(C3_MERGES):
        assert vc.step() is not None
    _check(vc, snap[C3_MERGES])
    vc.close()
