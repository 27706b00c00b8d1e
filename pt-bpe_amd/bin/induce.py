#!/usr/bin/env python
"""Tokenize new chains with a trained GeoBPE vocabulary on MI355X -- the caller
side of the reference's ``bin/induce.py`` (flags :34-51, main :141-239).

  * ``--src-pkl``: a ``bpe_iter=*.pkl`` checkpoint (this build's or the
    reference's own), read through geobpe.refpickle's whitelisted reader.
  * ``--data-dir``: an internal-coordinate corpus (.npz, geobpe.synth layout) or
    ``synthetic:N:LO:HI:SEED``; PDB featurisation is SURVEY.md §8(f) row 2.
  * The chains are tokenized by merge replay (geobpe.induce; the reference's
    BPE.tokenize does not run in the scoped mode): the trained
    merges in order, each applied to every occurrence greedily left to right.
  * Writes ``<save-dir>/utility.json`` (codebook utility of the new ids,
    induce.py:225-227) and ``<save-dir>/<src name>``: the source object with
    ``tokenizers`` replaced by the new ones, or appended with ``--append`` (and
    ``n`` turned into a list, induce.py:230-239).
Chains with a residue geometry outside the trained vocabulary, or values outside
the trained histogram range, raise ValueError (get_ind, bpe.py:1164-1189).

A checkpoint of the RMSD-partitioned mode (it holds ``_sphere_dict``) is induced the
reference's way instead: ``BPE.tokenize`` of every chain (bpe.py:1053-1140, here
geobpe.rmsd_bpe.RmsdBPE.tokenize on device NeRF / RMSD batches), then the same
utility.json and output pickle (induce.py:216-239).
"""
from __future__ import annotations

import argparse
import json
import os
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


def parse_args(argv=None):
    p = argparse.ArgumentParser(description="GeoBPE (MI355X) induction script")
    p.add_argument("--src-pkl", required=True)
    p.add_argument("--base-dir", type=str, default="./")
    p.add_argument("--save-dir")
    p.add_argument("--log-dir", type=str, default="logs")
    p.add_argument("--data-dir", required=True)
    p.add_argument("--toy", default=0, type=int)
    p.add_argument("--pad", default=512, type=int)
    p.add_argument("--processed", type=str2bool, default=False)
    p.add_argument("--debug", action="store_true")
    p.add_argument("--append", action="store_true", help="Whether to append to src-pkl")
    p.add_argument("--device", type=int, default=0)
    return p.parse_args(argv)


def main(argv=None) -> int:
    args = parse_args(argv)
    from geobpe import induce, refpickle
    from geobpe.bpe import get_codebook_utility

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from encode import load_corpus

    save_dir = args.save_dir or os.path.join(args.base_dir, "ckpts", str(time.time()))
    os.makedirs(save_dir, exist_ok=True)
    args_path = os.path.join(save_dir, "args.txt")
    if os.path.exists(args_path):  # validate_args_match (utils.py), skip auto / save_dir
        with open(args_path) as f:
            loaded = dict(line.rstrip("\n").split(": ", 1) for line in f if ": " in line)
        for k, v in sorted(vars(args).items()):
            if k not in ("save_dir", "device") and k in loaded and loaded[k] != str(v):
                raise SystemExit(f"argument mismatch for {k}: saved {loaded[k]!r} != current {v!r}")
    else:
        with open(args_path, "w") as f:
            for k, v in sorted(vars(args).items()):
                f.write(f"{k}: {v}\n")
    src_args = os.path.join(os.path.dirname(os.path.abspath(args.src_pkl)), "args.txt")
    if os.path.exists(src_args):
        with open(src_args) as f, open(os.path.join(save_dir, "orig_args.txt"), "w") as g:
            g.write(f.read())

    bpe = refpickle.load(args.src_pkl)
    if getattr(bpe, "_sphere_dict", None) is not None:
        return induce_rmsd(args, bpe, save_dir)
    B = int(bpe.bins[1])
    thr = {k: [tuple(p) for p in v] for k, v in bpe._thresholds[1].items()}
    corpus = load_corpus(args.data_dir, args.toy)
    t0 = time.time()
    eng = induce.induce(corpus, bpe._tokens, thr, B, device=args.device)
    start, ids, off = eng.segmentation()
    a, b, eoff = eng.events()
    enc, eoff_ids = eng.encode()
    sol = eng.sym_of_label
    nrows = len(corpus["row_off"]) - 1
    run = {"corpus": corpus, "fnames": [f"{args.data_dir}#{i}" for i in range(nrows)], "B": B,
           "thresholds": thr, "K0": eng.K0, "sym_of_label": sol, "seg_start": start, "seg_id": ids,
           "seg_off": off, "ev_a": a, "ev_b": b, "ev_off": eoff}
    toks, _ = refpickle.build_tokenizers(run)
    eng.close()
    vocab_size = len(bpe._tokens) + 3 * B
    utility = get_codebook_utility(enc, vocab_size)
    with open(os.path.join(save_dir, "utility.json"), "w") as f:
        json.dump(utility, f)
    if args.append:
        if not isinstance(bpe.n, list):
            bpe.n = [bpe.n]
        bpe.n.append(len(toks))
        bpe.tokenizers.extend(toks)
    else:
        bpe.tokenizers = toks
    out_path = os.path.join(save_dir, os.path.basename(args.src_pkl))
    tmp = out_path + ".tmp"
    with open(tmp, "wb") as f:
        refpickle.dump(bpe, f)
    os.replace(tmp, out_path)
    print(json.dumps({"out": os.path.abspath(out_path), "chains": nrows, "tokens": int(len(ids)),
                      "seconds": round(time.time() - t0, 3)} | utility))
    return 0


def induce_rmsd(args, obj, save_dir: str) -> int:
    """RMSD mode: the trained state from the checkpoint, BPE.tokenize per chain, the
    utility of quantize(t.tokenize()) over all chains, the output pickle."""
    from geobpe import refpickle
    from geobpe.bpe import get_codebook_utility
    from geobpe.rmsd_bpe import RmsdBPE
    from geobpe.synth import COLUMNS
    from encode import load_corpus

    corpus = load_corpus(args.data_dir, args.toy)
    bpe = RmsdBPE.from_checkpoint(obj, device=args.device)
    t0 = time.time()
    ro = corpus["row_off"]
    fnames = corpus.get("fnames")
    toks, ids, ntok = [], [], 0
    for i in range(len(ro) - 1):
        struct = {"angles": {c: corpus[c][ro[i]:ro[i + 1]] for c in COLUMNS},
                  "fname": fnames[i] if fnames is not None else f"{args.data_dir}#{i}"}
        t, _ = bpe.tokenize(struct)
        ids.append(bpe.quantize(t))
        ntok += len(t.bond_to_token)
        toks.append(RmsdBPE.tokenizer_record(t))
    utility = get_codebook_utility(np.array([x for q in ids for x in q], dtype=np.int64), bpe.vocab_size)
    with open(os.path.join(save_dir, "utility.json"), "w") as f:
        json.dump(utility, f)
    if args.append:
        if not isinstance(obj.n, list):
            obj.n = [obj.n]
        obj.n.append(len(toks))
        obj.tokenizers.extend(toks)
    else:
        obj.tokenizers = toks
    out_path = os.path.join(save_dir, os.path.basename(args.src_pkl))
    tmp = out_path + ".tmp"
    with open(tmp, "wb") as f:
        refpickle.dump(obj, f)
    os.replace(tmp, out_path)
    print(json.dumps({"out": os.path.abspath(out_path), "chains": len(toks), "tokens": ntok,
                      "seconds": round(time.time() - t0, 3)} | utility))
    return 0


if __name__ == "__main__":
    sys.exit(main())
