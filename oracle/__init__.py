"""CPU oracle for the GeoBPE merge loop -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of
``bench.py`` may import this package, and only as the checker / the timed CPU
baseline.  The product (``pt-bpe_amd/``) never imports it.

Parity status: PINNED.  ``tests/test_oracle_golden.py`` checks this oracle
against every fixture in ``tests/golden/`` -- thresholds, initial labels, merge
list (key string + count), vocab, final segmentation and encoded ids -- which
``tests/golden/make_golden.py`` produced by running the reference
(``foldingdiff/bpe.py``) in the build container.

Layers:
  prologue.py        numpy restatement of the thresholds / symbols / labels
                     (bpe.py:820-876, 138-394, 1164-1189; plotting.py:305-337)
  geobpe_oracle.c    C restatement of bin()/step()/quantize() (bpe.py:1431-1474,
                     1792-2166, 918-956), built into liboracle.so by the Makefile.
"""
from __future__ import annotations

import ctypes
import json
import os
import subprocess

import numpy as np

from . import prologue

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")
_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        P, I64, I32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32
        L.oracle_create.restype = P
        L.oracle_create.argtypes = [I64, P, P, P, P, I32, I32]
        L.oracle_error.argtypes = [P]
        L.oracle_bin.argtypes = [P]
        L.oracle_step.restype = I32
        L.oracle_step.argtypes = [P, ctypes.POINTER(I32), ctypes.POINTER(I32)]
        L.oracle_key_json.restype = I64
        L.oracle_key_json.argtypes = [P, I32, ctypes.c_char_p, I64]
        L.oracle_num_keys.restype = I64
        L.oracle_num_keys.argtypes = [P]
        L.oracle_vocab_size_tokens.restype = I64
        L.oracle_vocab_size_tokens.argtypes = [P]
        L.oracle_vocab_content.restype = I64
        L.oracle_vocab_content.argtypes = [P, I32, P]
        L.oracle_vocab_nres.restype = I32
        L.oracle_vocab_nres.argtypes = [P, I32]
        L.oracle_segmentation.restype = I64
        L.oracle_segmentation.argtypes = [P, P, P, P]
        L.oracle_encode.restype = I64
        L.oracle_encode.argtypes = [P, P, P]
        L.oracle_destroy.argtypes = [P]
        _lib = L
    return _lib


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


class OracleBPE:
    """Scoped-mode GeoBPE on the CPU: ``initialize()``, ``bin()``, ``step()``."""

    def __init__(self, corpus: dict, bins: int, cover: bool = False, thresholds=None, sym_of_label=None,
                 strategy: str = None):
        """``thresholds`` / ``sym_of_label``: a trained vocabulary's grid and
        residue labels (merge replay on new chains); default: from this corpus."""
        self.corpus = corpus
        self.cover = cover
        self.strategy = strategy
        self._given = (thresholds, sym_of_label)
        self.B = int(bins)
        self.row_off = np.ascontiguousarray(corpus["row_off"], dtype=np.int64)
        self._h = None

    def initialize(self):
        thr, sol = self._given
        self.thresholds = thr if thr is not None else prologue.thresholds(self.corpus, self.B, self.cover, self.strategy)
        self.rsym, self.gsym = prologue.symbols(self.corpus, self.thresholds, self.B)
        if sol is None:
            self.labels, self.sym_of_label = prologue.init_labels(self.rsym)
        else:
            self.sym_of_label = np.asarray(sol, dtype=np.int32)
            lab = {int(s): i for i, s in enumerate(self.sym_of_label)}
            missing = sorted(set(int(x) for x in np.unique(self.rsym)) - set(lab))
            if missing:
                raise ValueError(f"residue symbols {missing[:5]} are not in the trained vocabulary")
            self.labels = np.array([lab[int(x)] for x in self.rsym], dtype=np.int32)
        self.K0 = len(self.sym_of_label)
        self._keep = (self.row_off, self.rsym, self.gsym, self.labels)
        L = lib()
        if self._given[1] is None:
            self._h = L.oracle_create(len(self.row_off) - 1, _ptr(self.row_off), _ptr(self.rsym),
                                      _ptr(self.gsym), _ptr(self.labels), self.K0, self.B)
        else:
            L.oracle_create_vocab.restype = ctypes.c_void_p
            L.oracle_create_vocab.argtypes = [ctypes.c_int64] + [ctypes.c_void_p] * 4 + [ctypes.c_int32] * 2 + \
                [ctypes.c_void_p]
            self._h = L.oracle_create_vocab(len(self.row_off) - 1, _ptr(self.row_off), _ptr(self.rsym),
                                            _ptr(self.gsym), _ptr(self.labels), self.K0, self.B,
                                            _ptr(self.sym_of_label))
        if L.oracle_error(self._h):
            raise RuntimeError("oracle: inconsistent initial labels")
        self.merges = []  # [(key_json, count)]
        return self

    def bin(self):
        lib().oracle_bin(self._h)

    def step(self):
        c, k = ctypes.c_int32(0), ctypes.c_int32(0)
        n = lib().oracle_step(self._h, ctypes.byref(c), ctypes.byref(k))
        if n < 0:
            return None
        self.merges.append((self.key_json(k.value), c.value))
        return n

    def step_forced(self, L: int, g: int, R: int):
        """Merge replay: merge the content L ++ [g] ++ R next (its token id is
        consumed even if it does not occur).  Returns (new id, count)."""
        Lb = lib()
        Lb.oracle_step_forced.restype = ctypes.c_int32
        Lb.oracle_step_forced.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                          ctypes.POINTER(ctypes.c_int32)]
        c = ctypes.c_int32(0)
        n = Lb.oracle_step_forced(self._h, int(L), int(g), int(R), ctypes.byref(c))
        self.merges.append((None, c.value))
        return n, c.value

    def step_fast(self):
        """step() without rendering the key string (for timing)."""
        c, k = ctypes.c_int32(0), ctypes.c_int32(0)
        n = lib().oracle_step(self._h, ctypes.byref(c), ctypes.byref(k))
        return None if n < 0 else (n, c.value, k.value)

    def key_json(self, k: int) -> str:
        L = lib()
        m = L.oracle_key_json(self._h, k, None, 0)
        buf = ctypes.create_string_buffer(int(m) + 1)
        L.oracle_key_json(self._h, k, buf, m + 1)
        return buf.value.decode()

    @property
    def num_tokens_vocab(self) -> int:
        return int(lib().oracle_vocab_size_tokens(self._h))

    @property
    def vocab_size(self) -> int:
        return self.num_tokens_vocab + 3 * self.B

    def segmentation(self):
        L = lib()
        T = L.oracle_segmentation(self._h, None, None, None)
        start = np.empty(T, np.int32)
        ids = np.empty(T, np.int32)
        off = np.empty(len(self.row_off), np.int64)
        L.oracle_segmentation(self._h, _ptr(start), _ptr(ids), _ptr(off))
        return start, ids, off

    def encode(self):
        L = lib()
        T = L.oracle_encode(self._h, None, None)
        ids = np.empty(T, np.int32)
        off = np.empty(len(self.row_off), np.int64)
        L.oracle_encode(self._h, _ptr(ids), _ptr(off))
        return ids, off

    def events(self):
        """Merge events in iteration order: (a, b, iter_off) -- left / right token
        start slots of every merged occurrence; events of merge t are
        [iter_off[t], iter_off[t+1])."""
        L = lib()
        L.oracle_events.restype = ctypes.c_int64
        L.oracle_events.argtypes = [ctypes.c_void_p] * 4
        n = L.oracle_events(self._h, None, None, None)
        a = np.empty(n, np.int32)
        b = np.empty(n, np.int32)
        off = np.empty(len(self.merges) + 1, np.int64)
        L.oracle_events(self._h, _ptr(a), _ptr(b), _ptr(off))
        return a, b, off

    def vocab_content(self, v: int) -> np.ndarray:
        L = lib()
        m = L.oracle_vocab_content(self._h, v, None)
        out = np.empty(m, np.int32)
        L.oracle_vocab_content(self._h, v, _ptr(out))
        return out

    def vocab(self) -> dict:
        """`_tokens` as the reference holds it: residue tokens with bin-centre
        floats, merged tokens as json.loads(key)."""
        out = {}
        for v in range(self.K0):
            out[v] = prologue.residue_token_dict(int(self.sym_of_label[v]), self.thresholds, self.B)
        for i, (key, _) in enumerate(self.merges):
            out[self.K0 + i] = json.loads(key)
        return out

    def __del__(self):
        if self._h is not None and _lib is not None:
            _lib.oracle_destroy(self._h)
            self._h = None
