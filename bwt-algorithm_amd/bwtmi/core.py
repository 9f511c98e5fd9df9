"""BWTCore -- the reference's FM-index class (bwt.py:98-427) over the device
index built by libbwtmi (suffix array, BWT, C, Occ checkpoints, sampled SA
and 8-mer hash all constructed by HIP kernels on gfx950).  Host copies of
the arrays are fetched lazily, on first attribute access.
"""
from __future__ import annotations

import ctypes as C
from typing import Dict, List, Optional, Sequence, Tuple, Union

import numpy as np

from . import _lib
from ._lib import check, lib


class _LazyText:
    """`BWTCore.text` for an index built from bytes: the str is decoded on
    first use only (nothing on the CLI path reads it)."""

    def __init__(self, raw: bytes):
        self._raw, self._s = raw, None

    def _str(self) -> str:
        if self._s is None:
            self._s = self._raw.decode("latin-1")
        return self._s

    def __len__(self):
        return len(self._raw)

    def __str__(self):
        return self._str()

    def __eq__(self, other):
        return self._str() == (str(other) if isinstance(other, _LazyText) else other)

    def __hash__(self):
        return hash(self._str())

    def __getitem__(self, k):
        return self._str()[k]

    def __iter__(self):
        return iter(self._str())

    def __contains__(self, x):
        return x in self._str()

    def __getattr__(self, name):
        return getattr(self._str(), name)


class BWTCore:
    BASE_TO_BITS = {"A": 0, "C": 1, "G": 2, "T": 3, "N": 0}
    BITS_TO_BASE = {0: "A", 1: "C", 2: "G", 3: "T"}

    def __init__(self, text: Union[str, bytes], sa_sample_rate: int = 32, occ_sample_rate: int = 128,
                 device: Optional[int] = None, build_kmer: bool = True):
        # bytes are taken as the encoded text itself (no str is built: the CLI
        # hands over the loader's native contig bytes)
        raw = bytes(text) if isinstance(text, (bytes, bytearray, memoryview)) else None
        self.text = text if raw is None else _LazyText(raw)
        self.n = len(text)
        self.sa_sample_rate = sa_sample_rate
        self.occ_sample_rate = occ_sample_rate
        self.text_arr = np.frombuffer(raw if raw is not None else text.encode("utf-8"), dtype=np.uint8)
        self._ctx = _lib.ctx(device)
        self._h = C.c_void_p()
        buf = self.text_arr if self.text_arr.size else np.zeros(1, dtype=np.uint8)
        check(lib().bwtmi_index_build(self._ctx, buf.ctypes.data_as(C.c_void_p), self.text_arr.size,
                                      sa_sample_rate, occ_sample_rate, 0 if build_kmer else 1,
                                      C.byref(self._h)))
        totals = np.zeros(256, dtype=np.int64)
        cum = np.zeros(256, dtype=np.int64)
        check(lib().bwtmi_index_get_counts(self._h, totals.ctypes.data_as(C.c_void_p),
                                           cum.ctypes.data_as(C.c_void_p)))
        self._totals, self._C = totals, cum
        if raw is not None or text.isascii():
            # ASCII text (O(1) test on a CPython str): the characters are the
            # byte values the device histogram found (bwt.py:129)
            self.alphabet = [chr(c) for c in np.nonzero(totals)[0].tolist()]
        else:
            self.alphabet = sorted(set(text))
        self.char_to_code = {c: ord(c) for c in self.alphabet}
        self.code_to_char = {ord(c): c for c in self.alphabet}
        self.char_counts = {c: int(cum[ord(c)]) for c in self.alphabet if ord(c) < 256}
        self.char_totals = {c: int(totals[ord(c)]) for c in self.alphabet if ord(c) < 256}
        self.char_counts_code = {ord(k): v for k, v in self.char_counts.items()}
        self.char_totals_code = {ord(k): v for k, v in self.char_totals.items()}
        self._sa = self._bwt = self._occ = self._sampled = self._kmer = None

    def __del__(self):
        h = getattr(self, "_h", None)
        if h and _lib._lib is not None:
            _lib._lib.bwtmi_index_free(h)
            self._h = None

    # ---------------------------------------------------------------- arrays
    @property
    def suffix_array(self) -> np.ndarray:
        if self._sa is None:
            a = np.zeros(max(self.text_arr.size, 1), dtype=np.int32)
            check(lib().bwtmi_index_get_sa(self._h, a.ctypes.data_as(C.c_void_p)))
            self._sa = a[:self.text_arr.size]
        return self._sa

    @property
    def bwt_arr(self) -> np.ndarray:
        if self._bwt is None:
            a = np.zeros(max(self.text_arr.size, 1), dtype=np.uint8)
            check(lib().bwtmi_index_get_bwt(self._h, a.ctypes.data_as(C.c_void_p)))
            self._bwt = a[:self.text_arr.size]
        return self._bwt

    @property
    def occ_checkpoints(self) -> Dict[int, np.ndarray]:
        if self._occ is None:
            L = lib().bwtmi_index_occ_len(self._h)
            occ = {}
            if self.text_arr.size:
                for code in np.nonzero(self._totals)[0].tolist():
                    a = np.zeros(L, dtype=np.int32)
                    check(lib().bwtmi_index_get_occ(self._h, code, a.ctypes.data_as(C.c_void_p)))
                    occ[int(code)] = a
                for ch in self.alphabet:       # bwt.py:319-325
                    if ord(ch) not in occ:
                        occ[ord(ch)] = np.zeros(L, dtype=np.int32)
            self._occ = occ
        return self._occ

    @property
    def sampled_sa(self) -> Dict[int, int]:
        if self._sampled is None:
            m = lib().bwtmi_index_sampled_len(self._h)
            a = np.zeros(max(m, 1), dtype=np.int32)
            if m:
                check(lib().bwtmi_index_get_sampled(self._h, a.ctypes.data_as(C.c_void_p)))
            self._sampled = {i * self.sa_sample_rate: int(a[i]) for i in range(m)}
        return self._sampled

    def kmer_csr(self) -> Tuple[np.ndarray, np.ndarray]:
        m = lib().bwtmi_index_kmer_count(self._h)
        off = np.zeros(65537, dtype=np.int64)
        pos = np.zeros(max(m, 1), dtype=np.int32)
        check(lib().bwtmi_index_get_kmer(self._h, off.ctypes.data_as(C.c_void_p),
                                         pos.ctypes.data_as(C.c_void_p)))
        return off, pos[:m]

    @property
    def kmer_hash(self) -> Dict[int, List[int]]:
        if self._kmer is None:
            off, pos = self.kmer_csr()
            nz = np.nonzero(np.diff(off))[0]
            self._kmer = {int(c): pos[off[c]:off[c + 1]].tolist() for c in nz.tolist()}
        return self._kmer

    def get_kmer_positions(self, kmer: str) -> List[int]:
        """bwt.py:173-193 (including its direct lookup of k < 8 codes)."""
        if len(kmer) > 8 or not self.kmer_hash:
            return self.locate_positions(kmer)
        w = 0
        for b in kmer.upper():
            if b not in self.BASE_TO_BITS:
                return []
            w = (w << 2) | self.BASE_TO_BITS[b]
        return list(self.kmer_hash.get(w, []))

    def clear(self):
        self.text = ""
        self.text_arr = np.array([], dtype=np.uint8)
        self._sa = np.array([], dtype=np.int32)
        self._bwt = np.array([], dtype=np.uint8)
        self._sampled, self._occ = {}, {}
        self.char_counts, self.char_totals, self.alphabet = {}, {}, []
        self.char_to_code, self.code_to_char = {}, {}
        self.char_counts_code, self.char_totals_code = {}, {}
        if self._h and _lib._lib is not None:
            _lib._lib.bwtmi_index_free(self._h)
            self._h = None

    # ---------------------------------------------------------------- queries
    def rank(self, char: Union[str, int], pos: int) -> int:
        if pos <= 0:
            return 0
        pos = min(pos, self.n)
        code = ord(char) if isinstance(char, str) else int(char)
        cp = self.occ_checkpoints.get(code)
        if cp is None:
            return 0
        k = self.occ_sample_rate
        ci = pos // k
        base = int(cp[ci])
        if pos > ci * k:
            base += int(np.count_nonzero(self.bwt_arr[ci * k:pos] == code))
        return base

    @staticmethod
    def pack_patterns(patterns: Sequence[str]) -> Tuple[np.ndarray, np.ndarray]:
        """(concatenated bytes, offsets[n + 1]) for backward_search_packed."""
        enc = [p.encode("utf-8") for p in patterns]
        off = np.zeros(len(enc) + 1, dtype=np.int64)
        off[1:] = np.cumsum([len(e) for e in enc]) if enc else 0
        blob = np.frombuffer(b"".join(enc) or b"\0", dtype=np.uint8)
        return blob, off

    def backward_search_packed(self, blob: np.ndarray, off: np.ndarray) -> np.ndarray:
        npat = off.size - 1
        out = np.zeros((max(npat, 1), 2), dtype=np.int64)
        check(lib().bwtmi_backward_search_batch(self._ctx, self._h, blob.ctypes.data_as(C.c_void_p),
                                                off.ctypes.data_as(C.c_void_p), npat,
                                                out.ctypes.data_as(C.c_void_p)))
        return out[:npat]

    def backward_search_batch(self, patterns: Sequence[str]) -> np.ndarray:
        """Device batch of BWTCore.backward_search: int64[len(patterns), 2]."""
        return self.backward_search_packed(*self.pack_patterns(patterns))

    def backward_search(self, pattern: str) -> Tuple[int, int]:
        if not pattern:
            return (0, self.n - 1)
        if any(ch not in self.char_counts for ch in pattern):   # non-byte / absent symbols
            return (-1, -1)
        sp, ep = self.backward_search_batch([pattern])[0].tolist()
        return (int(sp), int(ep))

    def count_occurrences(self, pattern: str) -> int:
        sp, ep = self.backward_search(pattern)
        return 0 if sp == -1 else ep - sp + 1

    def locate_positions(self, pattern: str) -> List[int]:
        sp, ep = self.backward_search(pattern)
        if sp == -1:
            return []
        return sorted(self.suffix_array[sp:ep + 1].tolist())

    def _get_suffix_position(self, sa_index: int) -> int:
        return int(self.suffix_array[sa_index])

    def lcp_array(self) -> np.ndarray:
        """Kasai LCP over the index text (bwt.py:56-95) computed on the device."""
        out = np.zeros(max(self.text_arr.size, 1), dtype=np.int32)
        if self.text_arr.size:
            check(lib().bwtmi_index_lcp(self._ctx, self._h, out.ctypes.data_as(C.c_void_p)))
        return out[:self.text_arr.size]
