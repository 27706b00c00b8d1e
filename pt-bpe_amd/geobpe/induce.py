"""Merge replay: tokenize new chains with a trained GeoBPE vocabulary.

bin/induce.py of the reference loads a trained ``bpe_iter=*.pkl`` and tokenizes
new structures with ``BPE.tokenize`` (bin/induce.py:58-75,160-239); in the
scoped mode that method does not run.  This build
defines induction as the training loop with the argmax replaced by the trained
merge order: merge t is token K0 + t of the vocabulary, applied to every current
occurrence greedily left to right exactly as in training (bpe.py:1888-2014).  On
the training corpus the replay reproduces the training segmentation, token for
token (tests/test_gpu_parity.py).

The device side is the merge loop itself (k_select_replay instead of k_select,
geobpe_replay_load in include/geobpe.h).  This module derives, from a
vocabulary (``_thresholds``, ``_tokens``), the replay records: per merged token
its content hash (the polynomial of device.h over the interleaved residue /
junction symbols), its length and one split into two earlier tokens.
"""
from __future__ import annotations

import json

import numpy as np

M61 = (1 << 61) - 1
HP1 = 0x0A3B5C7D9E1F2437 % M61  # device.h content-hash bases
HP2 = 0x13579BDF2468ACE1 % M61
ANGLE_KEYS = ["tau", "CA:C:1N", "C:1N:1CA", "psi", "omega", "phi"]


def content_hash(seq) -> tuple:
    """H(s_0..s_{n-1}) = sum (s_i + 1) P^(n-1-i) mod 2^61-1 for both bases (device.h combine)."""
    h1 = h2 = 0
    for s in seq:
        h1 = (h1 * HP1 + s + 1) % M61
        h2 = (h2 * HP2 + s + 1) % M61
    return h1, h2


def _bin_of_centre(thr, v: float) -> int:
    for i, (s, e) in enumerate(thr):
        if sum((s, e)) / 2 == v:
            return i
    raise ValueError(f"{v} is not a bin centre of {thr}")


def residue_symbol(tok: dict, thr: dict, B: int) -> int:
    """Residue symbol of a residue token (bin-centre geometry, bpe.py:236-261)."""
    tau = _bin_of_centre(thr["tau"], tok["tau"][0])
    if "psi" not in tok:  # the last residue of a chain: only tau (+ two bonds)
        return B ** 3 + tau
    return tau * B * B + _bin_of_centre(thr["CA:C:1N"], tok["CA:C:1N"][0]) * B + _bin_of_centre(thr["psi"], tok["psi"][0])


def merged_content(tok: dict, B: int) -> tuple:
    """Interleaved content R0 G0 R1 ... R_{r-1} of a merged token (json.loads(key):
    bin indices)."""
    r = len(tok["tau"])
    last = len(tok["psi"]) == r - 1
    seq = []
    for j in range(r):
        if j == r - 1 and last:
            seq.append(B ** 3 + tok["tau"][j])
        else:
            seq.append(tok["tau"][j] * B * B + tok["CA:C:1N"][j] * B + tok["psi"][j])
        if j < r - 1:
            seq.append(tok["omega"][j] * B * B + tok["C:1N:1CA"][j] * B + tok["phi"][j])
    return tuple(seq)


def vocabulary(tokens: dict, thresholds: dict, B: int):
    """(sym_of_label, K0, contents) of a trained ``_tokens`` dict: residue tokens
    (bin-centre floats) first, then merged tokens (bin indices)."""
    ids = sorted(tokens)
    if ids != list(range(len(ids))):
        raise ValueError("token ids are not 0..K-1")
    sym_of_label, contents = [], []
    for v in ids:
        d = tokens[v]
        vals = [x for lst in d.values() for x in lst]
        merged = bool(vals) and all(isinstance(x, (int, np.integer)) for x in vals)
        if not merged:
            if contents and len(contents) > len(sym_of_label):
                raise ValueError(f"token {v}: residue token after merged tokens")
            s = residue_symbol(d, thresholds, B)
            sym_of_label.append(s)
            contents.append((s,))
        else:
            contents.append(merged_content(d, B))
    return np.array(sym_of_label, dtype=np.int32), len(sym_of_label), contents


def replay_records(contents, K0: int) -> dict:
    """Per merged token K0 + t: content hash, residues, and a split L ++ [g] ++ R
    into earlier tokens (the first split whose halves are both earlier tokens)."""
    first = {}
    for v in range(K0):
        first.setdefault(contents[v], v)
    M = len(contents) - K0
    rec = {k: np.zeros(M, dtype=np.uint64 if k in ("h1", "h2") else np.int32)
           for k in ("h1", "h2", "len", "idL", "g", "idR")}
    for t in range(M):
        v = K0 + t
        c = contents[v]
        r = (len(c) + 1) // 2
        split = None
        for i in range(1, r):
            a, b = first.get(c[: 2 * i - 1]), first.get(c[2 * i:])
            if a is not None and b is not None:
                split = (a, c[2 * i - 1], b)
                break
        if split is None:
            raise ValueError(f"token {v} is not a merge of two earlier tokens")
        h1, h2 = content_hash(c)
        rec["h1"][t], rec["h2"][t], rec["len"][t] = h1, h2, r
        rec["idL"][t], rec["g"][t], rec["idR"][t] = split
        first.setdefault(c, v)
    return rec


def merge_keys_of(contents, K0: int, B: int):
    """Key strings of the merged tokens (json.dumps(json.loads(key), sort_keys=True))."""
    from .refpickle import span_key
    out = []
    for c in contents[K0:]:
        rs = np.array(c[0::2])
        gs = np.array(list(c[1::2]) + [-1])
        last = rs[-1] >= B ** 3
        out.append(span_key(rs, gs, 0, len(rs) - 1, bool(last), B))
    return out


def induce(corpus: dict, tokens: dict, thresholds: dict, B: int, device: int = 0, record_events: bool = True):
    """Tokenize ``corpus`` with the trained vocabulary on the GPU; returns the
    engine after the replay (segmentation(), encode(), events())."""
    from .engine import GeoBPEEngine
    sym_of_label, K0, contents = vocabulary(tokens, thresholds, B)
    rec = replay_records(contents, K0)
    eng = GeoBPEEngine(corpus, B, device=device)
    eng.initialize(thresholds=thresholds, sym_of_label=sym_of_label)
    eng.bin()
    eng.replay_load(rec)
    if record_events:
        eng.record_events(True)
    M = len(contents) - K0
    if M:
        eng.run(M)
    return eng


def tokens_from_json(d: dict) -> dict:
    return {int(k): v for k, v in d.items()}


def dumps_key(tok: dict) -> str:
    return json.dumps(tok, sort_keys=True)
