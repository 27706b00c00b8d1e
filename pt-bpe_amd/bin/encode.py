#!/usr/bin/env python
"""GeoBPE training driver on MI355X -- the caller side of the hot path,
mirroring the reference's ``bin/encode.py`` (flags :106-167, loop :371-427).

Differences (all outside SURVEY.md §8's hot path):
  * ``--data-dir`` takes a directory of PDB files (geobpe.pdb: C++ backbone
    reader + HIP featurisation, the dataset's filters and shuffle), an
    internal-coordinate corpus (``.npz`` in the geobpe.synth layout) or
    ``synthetic:N:LO:HI:SEED``.
  * stats JSON carries K, L, bpr and the codebook utility (encode.py:408-420);
    bb_rmsd / lddt need the coordinate stack (esm ProteinChain) and are omitted.
  * checkpoints are ``bpe_iter={t}.pkl`` in the reference's pickle format
    (geobpe.refpickle: a foldingdiff.bpe.BPE object that bin/train.py,
    bin/predict.py, bin/induce.py and the reference's resume load unchanged);
    ``--ckpt-format json`` writes the bare merge list instead.  Resume (either
    format, the reference's own pkl files included) reads the merge list, re-runs
    that many merges on the device and checks them against it.
  * ``--run-chunk M`` (ours): merges issued per device call between host
    syncs; the reference steps one at a time.  Outputs do not depend on it.

Out-of-scope flag values (res-init false, --glue-opt-method each, glue-opt
without --p-min-size, uniform bins with free bonds) raise NotImplementedError
from geobpe.bpe.BPE before any work starts.  With --p-min-size < inf the run is
the RMSD-partitioned mode (geobpe.rmsd_bpe.RmsdBPE); --glue-opt true with
--glue-opt-method all runs glue_opt_all after initialize (encode.py:331-332) and
the per-step re-optimisation, on the device.
"""
from __future__ import annotations

import argparse
import glob
import json
import logging
import os
import re
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def str2bool(v):
    if isinstance(v, bool):
        return v
    if v.lower() in ("yes", "true", "t", "y", "1"):
        return True
    if v.lower() in ("no", "false", "f", "n", "0"):
        return False
    raise argparse.ArgumentTypeError("Boolean value expected.")


def str2dict(v):
    if not re.match(r"\d+-\d+(?::\d+-\d+)*$", v):
        raise argparse.ArgumentTypeError("Wrong format, see help.")
    return {int(a): int(b) for a, b in re.findall(r"(\d+)-(\d+)", v)}


def int_or_inf(x):
    if x.lower() in ("inf", "infinity"):
        return float("inf")
    try:
        return int(x)
    except ValueError:
        raise argparse.ArgumentTypeError(f"'{x}' is not an integer or 'inf'")


def parse_args(argv=None):
    p = argparse.ArgumentParser(description="GeoBPE (MI355X) BPE script")
    p.add_argument("--auto", action="store_true")
    p.add_argument("--base-dir", type=str, default="./")
    p.add_argument("--save-dir", type=str)
    p.add_argument("--log-dir", type=str, default="logs")
    p.add_argument("--data-dir", type=str, default="synthetic:1000:40:300:0",
                   help="a directory of PDB files, a corpus .npz (geobpe.synth layout) or synthetic:N:LO:HI:SEED")
    p.add_argument("--toy", type=int, default=0, help="number of chains; 0 for all")
    p.add_argument("--res-init", type=str2bool, default=True)
    p.add_argument("--free-bonds", type=str2bool, default=False)
    p.add_argument("--bin-strategy", default="histogram", choices=["histogram", "histogram-cover", "uniform"])
    p.add_argument("--bins", type=str2dict, default="1-10")
    p.add_argument("--p-min-size", type=int_or_inf, default=float("inf"))
    p.add_argument("--max-iter", type=int, default=10000)
    p.add_argument("--num-p", type=str2dict, default="1-3",
                   help="k-medoids partitions per token size (RMSD mode, --p-min-size < inf)")
    p.add_argument("--max-num-strucs", type=int, default=500)
    p.add_argument("--rmsd-super-res", type=str2bool, default=False)
    p.add_argument("--glue-opt", type=str2bool, default=False)
    p.add_argument("--glue-opt-prior", type=float, default=0.0)
    p.add_argument("--glue-opt-every", type=int, default=10)
    p.add_argument("--glue-opt-method", choices=["each", "all"], default="each",
                   help="RMSD mode: 'all' runs (device L-BFGS); 'each' is not built")
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--save-every", type=int, default=10)
    p.add_argument("--run-chunk", type=int, default=0, help="merges per device call (0: = save-every)")
    p.add_argument("--device", type=int, default=0)
    p.add_argument("--ckpt-format", choices=["pkl", "json"], default="pkl")
    p.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                   help="under torchrun (WORLD_SIZE > 1): rows sharded over the ranks, RCCL by default")
    return p.parse_args(argv)


def load_corpus(spec: str, toy: int = 0) -> dict:
    from geobpe import synth
    if spec.startswith("synthetic:"):
        n, lo, hi, seed = (int(x) for x in spec.split(":")[1:5])
        corpus = synth.make_corpus(synth.make_lengths(n, lo, hi, seed=seed), seed=seed)
    elif os.path.isdir(spec):  # a directory of PDB files (scripts/encode.sh, config 1)
        from geobpe import pdb
        corpus, fnames = pdb.load_pdb_dir(spec, toy=toy)
        corpus["fnames"] = fnames
        return corpus
    else:
        corpus = synth.load_corpus(spec)
    if toy:
        from geobpe.dist import slice_corpus
        corpus = slice_corpus(corpus, 0, min(toy, len(corpus["row_off"]) - 1))
    return corpus


def stats(bpe):
    """The stats json (encode.py:364,417); multi-GPU: None on ranks other than 0."""
    from geobpe.bpe import get_codebook_utility
    enc = bpe.encode_all()
    cap = bpe.capacity(tokenizer=True)
    if enc is None:
        return None
    ids, off = enc
    ntok = (np.diff(off) + 3) // 4
    N = len(ntok)
    L = float(np.mean(ntok)) if N else 0.0
    K = len(bpe._tokens)
    return {"K": K, "L": L, "bpr": cap / (N * L) if N else 0.0} | \
        get_codebook_utility(ids, bpe.vocab_size)


def _saved_keys(path: str):
    """Merge key strings of a checkpoint, or None if it is incomplete."""
    if path.endswith(".json"):
        try:
            with open(path) as fh:
                return [m[0] for m in json.load(fh)["merges"]]
        except (OSError, ValueError, KeyError):
            return None
    from geobpe import refpickle
    if not refpickle.is_complete(path):  # encode.py:183-200 skips incomplete pickles
        return None
    obj = refpickle.load(path)
    if getattr(obj, "_sphere_dict", None) is not None:  # RMSD mode: one _sphere_dict key per step()
        return rmsd_merge_keys(obj)
    return refpickle.merge_keys(obj)


def rmsd_merge_keys(bpe) -> list:
    """The RMSD mode's merge keys in merge order: _sphere_dict without the residue
    partitions' keys (bpe.py:333-339, 1780)."""
    from geobpe.rmsd_bpe import RES_SPHERE_KEY
    res = set(RES_SPHERE_KEY.values())
    return [k for k in getattr(bpe, "_sphere_dict", {}) if k not in res]


def latest_checkpoint(save_dir: str):
    best, path, keys = -1, None, None
    for f in glob.glob(os.path.join(save_dir, "bpe_iter=*")):
        m = re.match(r"bpe_iter=(\d+)\.(pkl|json)$", os.path.basename(f))
        if not m or int(m.group(1)) <= best:
            continue
        k = _saved_keys(f)
        if k is not None:
            best, path, keys = int(m.group(1)), f, k
    return best, path, keys


def main(argv=None) -> int:
    args = parse_args(argv)
    if not args.save_dir:
        if not args.auto:
            raise SystemExit("--save-dir or --auto is required")
        args.save_dir = os.path.join(args.base_dir, "ckpts", str(time.time()))
    os.makedirs(args.save_dir, exist_ok=True)
    args_path = os.path.join(args.save_dir, "args.txt")
    skip = {"auto", "save_dir", "max_iter", "run_chunk", "device", "ckpt_format", "dist_backend"}
    if os.path.exists(args_path):  # validate_args_match (utils.py)
        with open(args_path) as f:
            loaded = dict(line.rstrip("\n").split(": ", 1) for line in f if ": " in line)
        for k, v in sorted(vars(args).items()):
            if k not in skip and k in loaded and loaded[k] != str(v):
                raise SystemExit(f"argument mismatch for {k}: saved {loaded[k]!r} != current {v!r}")
    else:
        with open(args_path, "w") as f:
            for k, v in sorted(vars(args).items()):
                f.write(f"{k}: {v}\n")
    os.makedirs(args.log_dir, exist_ok=True)
    logging.basicConfig(filename=os.path.join(args.log_dir, "encode.log"), level=logging.INFO)
    log = logging.getLogger("geobpe.encode")
    log.info(args)

    from geobpe.bpe import BPE
    rmsd_mode = args.p_min_size != float("inf")
    corpus = load_corpus(args.data_dir, args.toy)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    group, rank, shard, device = None, 0, corpus, args.device
    if world > 1:  # one process per GPU (torchrun): contiguous row blocks, deltas exchanged per merge
        import torch
        import torch.distributed as dist
        from geobpe.dist import TorchGroup, shard_rows, slice_corpus
        rank = int(os.environ["RANK"])
        device = int(os.environ.get("LOCAL_RANK", "0")) if args.dist_backend == "nccl" else args.device
        torch.cuda.set_device(device)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", device))
        else:
            dist.init_process_group("gloo")
        lo, hi = shard_rows(corpus["row_off"], world)[rank]
        shard = slice_corpus({k: v for k, v in corpus.items() if k != "fnames"}, lo, hi)
        group = TorchGroup(int(shard["row_off"][-1]), device=device)
    bpe = BPE(shard, bins=args.bins, bin_strategy=args.bin_strategy, save_dir=args.save_dir,
              res_init=args.res_init, std_bonds=not args.free_bonds,
              rmsd_partition_min_size=args.p_min_size, glue_opt=args.glue_opt, glue_opt_prior=args.glue_opt_prior,
              glue_opt_every=args.glue_opt_every, glue_opt_method=args.glue_opt_method, seed=args.seed,
              num_partitions=args.num_p, max_num_strucs=args.max_num_strucs, rmsd_super_res=args.rmsd_super_res,
              device=device, record_tree=args.ckpt_format == "pkl", group=group,
              global_corpus=corpus if group is not None else None)
    t0 = time.time()
    bpe.initialize()
    if args.glue_opt and args.glue_opt_method == "all":  # encode.py:331-332
        bpe.glue_opt_all()
    st = stats(bpe)  # (every rank takes part in the gather; rank 0 writes)
    if rank == 0:
        with open(os.path.join(args.save_dir, "initial_stats=-1.json"), "w") as f:
            json.dump(st, f)
    bpe.bin()
    log.info("initialize+bin %.3fs", time.time() - t0)

    start, ck, keys = latest_checkpoint(args.save_dir)
    if ck is not None:  # resume: re-run the saved number of merges, then check them against the file
        if rmsd_mode:  # a step() may merge more than once there (recurring keys, bpe.py:2164-2166)
            got = (lambda: rmsd_merge_keys(bpe)) if ck.endswith(".pkl") else (lambda: [m[0] for m in bpe.merges])
            while len(got()) < len(keys) and bpe.run(1):
                pass
            merged = got()
        else:
            bpe.run(len(keys))
            merged = [m[0] for m in bpe.merges]
        if merged != keys:
            raise SystemExit(f"replay of {ck} diverged from the saved merge list")
        log.info("resumed from %s at iter=%d", ck, start)

    chunk = args.run_chunk or args.save_every
    t = start + 1
    while t < args.max_iter:
        # next save point: t with t % save_every == 0 (encode.py:403)
        nxt = min(args.max_iter - 1, t + (-t) % args.save_every, t + chunk - 1)
        n = nxt - t + 1
        got = bpe.run(n)
        if got < n:
            log.info("no pairs left after %d merges", bpe._step)
            break
        t = nxt
        if t % args.save_every == 0:
            st = stats(bpe)
            if rank == 0:
                with open(os.path.join(args.save_dir, f"stats={t}.json"), "w") as f:
                    json.dump(st, f)
            if args.ckpt_format == "pkl":
                bpe.save_checkpoint(os.path.join(args.save_dir, f"bpe_iter={t}.pkl"))
            elif rank == 0:
                tmp = os.path.join(args.save_dir, f".bpe_iter={t}.json.tmp")
                with open(tmp, "w") as f:
                    json.dump({"iter": t, "merges": [list(m) for m in bpe.merges],
                               "args": {k: str(v) for k, v in vars(args).items()}}, f)
                os.replace(tmp, os.path.join(args.save_dir, f"bpe_iter={t}.json"))
        t += 1
    log.info("done: %d merges, vocab_size %d", bpe._step, bpe.vocab_size)
    if rank == 0:
        print(json.dumps({"merges": bpe._step, "vocab_size": bpe.vocab_size, "ranks": world,
                          "seconds": time.time() - t0}))
    bpe.close()
    if group is not None:
        import torch.distributed as dist
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
