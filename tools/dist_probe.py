"""N ranks of the sharded GeoBPE protocol on ONE GPU (gloo exchange): merge list
vs a single-engine run, and the time per merge of the multi-rank loop.

  python tools/dist_probe.py [world] [chains] [merges]
"""
import os
import socket
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "pt-bpe_amd"))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def worker(rank, world, port, n, merges, q):
    import torch
    import torch.distributed as dist
    from geobpe import synth
    from geobpe.dist import TorchGroup, shard_rows, slice_corpus
    from geobpe.engine import GeoBPEEngine
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    corpus = synth.make_corpus(synth.make_lengths(n, 40, 560, seed=0), seed=0)
    lo, hi = shard_rows(corpus["row_off"], world)[rank]
    shard = slice_corpus(corpus, lo, hi)
    g = TorchGroup(int(shard["row_off"][-1]), device=0)
    e = GeoBPEEngine(shard, 5, device=0, group=g).initialize()
    e.bin()
    e.run(10)
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    done = e.run(merges)
    torch.cuda.synchronize()
    dist.barrier()
    T = time.perf_counter() - t0
    q.put((rank, done, T, e.merge_keys()))
    dist.destroy_process_group()


def main():
    import multiprocessing as mp
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 10000
    merges = int(sys.argv[3]) if len(sys.argv) > 3 else 200
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=worker, args=(r, world, port, n, merges, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=600) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    import torch  # noqa: F401
    from geobpe import synth
    from geobpe.engine import GeoBPEEngine
    corpus = synth.make_corpus(synth.make_lengths(n, 40, 560, seed=0), seed=0)
    e = GeoBPEEngine(corpus, 5, device=0).initialize()
    e.bin()
    e.run(10 + merges)
    ref = e.merge_keys()
    same = all(r[3] == ref for r in res)
    T = max(r[2] for r in res)
    print(f"world {world} chains {n}: merges {res[0][1]} in {T:.3f}s = {res[0][1] / T:.0f} merges/s "
          f"({1e6 * T / max(res[0][1], 1):.0f} us/merge); merge list == 1-GPU: {same}", flush=True)
    if not same:
        sys.exit(1)


if __name__ == "__main__":
    main()
