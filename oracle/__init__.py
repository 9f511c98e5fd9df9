"""CPU ORACLE for the bwt-algorithm hot path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this package, and only as the checker / CPU baseline.  The
product (``bwt-algorithm_amd``) must never import it: a product path that
routed through the oracle would void every parity claim.

Contents
--------
* ``liboracle.so`` (``bwt_oracle.c``): plain-C restatement of the integer
  kernels -- strict adjacency scan (bwt.py:1891-2001), suffix array by prefix
  doubling (bwt.py:228-264), BWT (266-274), C table (276-286), Occ
  checkpoints (288-326), rank/backward search (335-389), 8-mer hash
  (138-171), Kasai LCP (78-95).
* ``post.py``: pure-Python restatement of the record construction and the
  sequential post-processing / writers (bwt.py:3402-3944, 3995-4198).

Pinning: every function is checked against the reference's own outputs
(tests/golden, produced by tests/golden/make_goldens.py which imports
/root/reference in the build container) by tests/test_oracle.py.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from typing import List, Tuple

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def build() -> str:
    """Compile liboracle.so (gcc) in-tree; returns its path."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return os.path.join(_HERE, "liboracle.so")


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            build()
        L = C.CDLL(path)
        p = C.c_void_p
        L.orc_strict_scan.restype = C.c_int64
        L.orc_strict_scan.argtypes = [p, C.c_int64, C.c_int32, C.c_int32, C.c_int32, C.c_int32,
                                      C.c_int32, C.POINTER(C.POINTER(C.c_int64))]
        L.orc_free.argtypes = [p]
        L.orc_suffix_array.argtypes = [p, C.c_int64, p]
        L.orc_set_sa_threads.argtypes = [C.c_int32]
        L.orc_bwt.argtypes = [p, C.c_int64, p, p]
        L.orc_char_counts.argtypes = [p, C.c_int64, p, p]
        L.orc_occ_len.restype = C.c_int64
        L.orc_occ_len.argtypes = [C.c_int64, C.c_int32]
        L.orc_occ.argtypes = [p, C.c_int64, C.c_int32, C.c_uint8, p]
        L.orc_backward_search.argtypes = [p, C.c_int64, C.c_int32, p, p, p, p, C.c_int64,
                                          C.POINTER(C.c_int64), C.POINTER(C.c_int64)]
        L.orc_kmer_csr.restype = C.c_int64
        L.orc_kmer_csr.argtypes = [p, C.c_int64, C.c_int32, p, p]
        L.orc_kasai.argtypes = [p, C.c_int64, p, p]
        _LIB = L
    return _LIB


def _u8(x) -> np.ndarray:
    if isinstance(x, (bytes, bytearray)):
        return np.frombuffer(bytes(x), dtype=np.uint8)
    if isinstance(x, str):
        return np.frombuffer(x.encode("utf-8"), dtype=np.uint8)
    return np.ascontiguousarray(x, dtype=np.uint8)


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


def strict_scan(text, min_unit: int = 1, max_unit: int = 120, max_mismatch: int = 0,
                min_copies: int = 3, threads: int = 0) -> np.ndarray:
    """Raw hits of find_long_unit_repeats_strict as int64[k,5] rows
    (start, end, unit_len, prim_len, copies), reference emission order."""
    t = _u8(text)
    out = C.POINTER(C.c_int64)()
    k = lib().orc_strict_scan(_ptr(t), len(t), min_unit, max_unit, max_mismatch, min_copies,
                              threads, C.byref(out))
    if k < 0:
        raise ValueError("bad strict-scan arguments")
    if k == 0:
        if out:
            lib().orc_free(out)
        return np.zeros((0, 5), dtype=np.int64)
    arr = np.ctypeslib.as_array(out, shape=(k * 5,)).copy().reshape(k, 5)
    lib().orc_free(out)
    return arr


def effective_max_unit(seq_len: int, min_copies: int = 3, max_unit_len: int = 120) -> int:
    """U used by _process_chromosome_worker (bwt.py:3095-3098)."""
    return max(max_unit_len, min(seq_len // min_copies, 1000))


class Index:
    """Reference-equivalent BWTCore arrays (text must include the sentinel)."""

    def __init__(self, text, sa_sample_rate: int = 32, occ_sample_rate: int = 128, k: int = 8,
                 threads: int = 1):
        """threads > 1 sorts each prefix-doubling round on that many threads
        (same order: the sort key is a total order)."""
        t = _u8(text)
        self.text = t
        n = len(t)
        self.n = n
        L = lib()
        self.sa = np.zeros(n, dtype=np.int32)
        L.orc_set_sa_threads(threads)
        try:
            L.orc_suffix_array(_ptr(t), n, _ptr(self.sa))
        finally:
            L.orc_set_sa_threads(1)
        self.bwt = np.zeros(n, dtype=np.uint8)
        L.orc_bwt(_ptr(t), n, _ptr(self.sa), _ptr(self.bwt))
        self.totals = np.zeros(256, dtype=np.int64)
        self.C = np.zeros(256, dtype=np.int64)
        L.orc_char_counts(_ptr(t), n, _ptr(self.totals), _ptr(self.C))
        self.occ_rate = occ_sample_rate
        olen = L.orc_occ_len(n, occ_sample_rate) if n else 0
        self.occ = np.zeros((256, max(olen, 1)), dtype=np.int32)
        for c in np.nonzero(self.totals)[0]:
            row = np.zeros(olen, dtype=np.int32)
            L.orc_occ(_ptr(self.bwt), n, occ_sample_rate, int(c), _ptr(row))
            self.occ[c, :olen] = row
        self.sampled_sa = {i: int(self.sa[i]) for i in range(0, n, sa_sample_rate)}
        self.k = k
        self.kmer_offsets = np.zeros((1 << (2 * k)) + 1, dtype=np.int64)
        self.kmer_pos = np.zeros(max(n, 1), dtype=np.int32)
        m = L.orc_kmer_csr(_ptr(t), n, k, _ptr(self.kmer_offsets), _ptr(self.kmer_pos))
        self.kmer_pos = self.kmer_pos[:m].copy()

    def alphabet(self) -> List[int]:
        return [int(c) for c in np.nonzero(self.totals)[0]]

    def backward_search(self, pattern) -> Tuple[int, int]:
        p = _u8(pattern)
        sp, ep = C.c_int64(), C.c_int64()
        lib().orc_backward_search(_ptr(self.bwt), self.n, self.occ_rate, _ptr(self.occ),
                                  _ptr(self.totals), _ptr(self.C), _ptr(p), len(p),
                                  C.byref(sp), C.byref(ep))
        return int(sp.value), int(ep.value)

    def kmer_positions(self, code: int) -> List[int]:
        return self.kmer_pos[self.kmer_offsets[code]:self.kmer_offsets[code + 1]].tolist()

    def lcp(self) -> np.ndarray:
        out = np.zeros(self.n, dtype=np.int32)
        lib().orc_kasai(_ptr(self.text), self.n, _ptr(self.sa), _ptr(out))
        return out
