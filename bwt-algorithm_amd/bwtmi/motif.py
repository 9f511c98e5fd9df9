"""MotifUtils -- the reference's motif helper namespace (bwt.py:675-1381).

Small string helpers are plain Python (they are called per motif, not per
base).  The banded per-copy alignment (`align_repeat_region`, the one heavy
helper) runs in the native library, the same code the post-processing uses.
"""
from __future__ import annotations

import ctypes as C
import math
from collections import Counter
from dataclasses import dataclass
from itertools import product
from typing import Dict, Iterator, List, Optional, Tuple

import numpy as np

from ._lib import lib

_COMP = {"A": "T", "T": "A", "C": "G", "G": "C", "N": "N"}
_TRANSITIONS = {("A", "G"), ("G", "A"), ("C", "T"), ("T", "C")}


@dataclass
class RepeatAlignmentSummary:          # bwt.py:661-674
    consensus: str
    motif_len: int
    copies: int
    consumed_length: int
    mismatch_rate: float
    max_errors_per_copy: int
    variations: List[str]
    copy_sequences: List[str]
    total_insertions: int
    total_deletions: int
    error_counts: List[int]


def _rotations(s: str):
    return (s[i:] + s[:i] for i in range(len(s)))


class MotifUtils:
    @staticmethod
    def get_canonical_motif(motif: str) -> str:
        return min(_rotations(motif)) if motif else motif

    @staticmethod
    def reverse_complement(seq: str) -> str:
        return "".join(_COMP.get(b, b) for b in seq[::-1])

    @staticmethod
    def get_canonical_motif_stranded(motif: str) -> Tuple[str, str]:
        if not motif:
            return motif, "+"
        fwd = min(_rotations(motif))
        rev = min(_rotations(MotifUtils.reverse_complement(motif)))
        return (fwd, "+") if fwd <= rev else (rev, "-")

    @staticmethod
    def is_primitive_motif(motif: str) -> bool:
        n = len(motif)
        return not any(n % p == 0 and motif[:p] * (n // p) == motif for p in range(1, n))

    @staticmethod
    def calculate_entropy(seq: str) -> float:
        if not seq:
            return 0.0
        n = len(seq)
        h = 0.0
        for c in Counter(seq).values():
            p = c / n
            h -= p * np.log2(p)
        return h

    @staticmethod
    def is_transition(base1: str, base2: str) -> bool:
        return base1 == base2 or (base1, base2) in _TRANSITIONS

    @staticmethod
    def hamming_distance(s1: str, s2: str) -> int:
        if len(s1) != len(s2):
            return max(len(s1), len(s2))
        return sum(a != b for a, b in zip(s1, s2))

    @staticmethod
    def hamming_distance_array(arr1: np.ndarray, arr2: np.ndarray) -> int:
        if arr1.size != arr2.size:
            return max(arr1.size, arr2.size)
        return int(np.count_nonzero(arr1 != arr2))

    @staticmethod
    def count_transversions_array(arr1: np.ndarray, arr2: np.ndarray) -> int:
        if arr1.size != arr2.size:
            return max(arr1.size, arr2.size)
        n = 0
        for b1, b2 in zip(arr1.tolist(), arr2.tolist()):
            if b1 != b2:
                c1 = chr(b1) if 65 <= b1 <= 84 else "N"
                c2 = chr(b2) if 65 <= b2 <= 84 else "N"
                n += not MotifUtils.is_transition(c1, c2)
        return n

    @staticmethod
    def edit_distance(a: str, b: str) -> int:
        if not a:
            return len(b)
        if not b:
            return len(a)
        prev = list(range(len(b) + 1))
        for i, ca in enumerate(a, 1):
            cur = [i] + [0] * len(b)
            for j, cb in enumerate(b, 1):
                cur[j] = min(prev[j] + 1, cur[j - 1] + 1, prev[j - 1] + (ca != cb))
            prev = cur
        return prev[-1]

    @staticmethod
    def smallest_period_str(s: str) -> int:
        n = len(s)
        for p in range(1, n + 1):
            if n % p == 0 and s == s[:p] * (n // p):
                return p
        return n

    @staticmethod
    def align_repeat_region(sequence: str, start: int, end: int, motif_template: str,
                            mismatch_fraction: float = 0.1, max_indel: Optional[int] = None,
                            min_copies: int = 3) -> Optional[RepeatAlignmentSummary]:
        if not motif_template or not sequence:
            return None
        seq = sequence.encode("latin-1", errors="replace")
        tmpl = motif_template.encode("latin-1", errors="replace")
        ints = (C.c_int64 * 8)()
        mm = C.c_double()
        cons = C.create_string_buffer(len(tmpl) + 1)
        var, cl, ce = C.c_void_p(), C.c_void_p(), C.c_void_p()
        rc = lib().bwtmi_align_region(seq, len(seq), start, end, tmpl, len(tmpl), mismatch_fraction,
                                      -1 if max_indel is None else max_indel, min_copies, ints,
                                      C.byref(mm), cons, C.byref(var), C.byref(cl), C.byref(ce))
        if rc < 0:
            from ._lib import check
            check(rc)
        if rc == 0:
            return None
        try:
            copies = ints[0]
            variations = C.string_at(var).decode() if var else ""
            lens = np.ctypeslib.as_array(C.cast(cl, C.POINTER(C.c_int64)), shape=(copies,)).tolist()
            errs = np.ctypeslib.as_array(C.cast(ce, C.POINTER(C.c_int64)), shape=(copies,)).tolist()
        finally:
            for p in (var, cl, ce):
                if p:
                    lib().bwtmi_free(p)
        seqs, pos = [], max(0, start)
        for ln in lens:
            seqs.append(sequence[pos:pos + ln])
            pos += ln
        return RepeatAlignmentSummary(
            consensus=cons.raw[:ints[1]].decode("latin-1"), motif_len=ints[1], copies=copies,
            consumed_length=ints[2], mismatch_rate=mm.value, max_errors_per_copy=ints[3],
            variations=variations.split(";") if variations else [], copy_sequences=seqs,
            total_insertions=ints[4], total_deletions=ints[5], error_counts=errs)

    @staticmethod
    def build_consensus_motif(sequences: List[str]) -> Tuple[str, float]:
        if not sequences:
            return "", 0.0
        if len(sequences) == 1:
            return sequences[0], 0.0
        m = len(sequences[0])
        out, mism = [], 0
        for pos in range(m):
            col = [s[pos] for s in sequences if pos < len(s)]
            if not col:
                out.append("N")
                continue
            top = Counter(col).most_common(1)[0][0]
            out.append(top)
            mism += len(col) - col.count(top)
        tot = len(sequences) * m
        return "".join(out), (mism / tot if tot > 0 else 0.0)

    @staticmethod
    def build_consensus_motif_array(text_arr: np.ndarray, start: int, motif_len: int,
                                    n_copies: int) -> Tuple[np.ndarray, float, int]:
        if n_copies == 0 or motif_len == 0:
            return np.array([], dtype=np.uint8), 0.0, 0
        copies = []
        for i in range(n_copies):
            a = start + i * motif_len
            if a + motif_len > text_arr.size:
                break
            copies.append(text_arr[a:a + motif_len])
        if not copies:
            return np.array([], dtype=np.uint8), 0.0, 0
        block = np.stack(copies)
        cons = np.zeros(motif_len, dtype=np.uint8)
        for p in range(motif_len):
            vals, cnt = np.unique(block[:, p], return_counts=True)
            cons[p] = vals[np.argmax(cnt)]     # ties -> smallest byte
        per = np.count_nonzero(block != cons[None, :], axis=1)
        return cons, float(per.sum()) / (len(copies) * motif_len), int(per.max())

    @staticmethod
    def summarize_variations_array(text_arr: np.ndarray, start: int, end: int, motif_len: int,
                                   consensus_arr: np.ndarray) -> List[str]:
        if text_arr.size == 0 or motif_len <= 0:
            return []
        seq = text_arr.tobytes().decode("ascii", errors="replace")
        start = max(0, start)
        end = min(len(seq), end if end > start else len(seq))
        if end <= start:
            return []
        tmpl = (consensus_arr.tobytes().decode("ascii", errors="replace") if consensus_arr.size
                else seq[start:start + motif_len])
        s = MotifUtils.align_repeat_region(seq, start, end, tmpl, mismatch_fraction=0.1, min_copies=1)
        return s.variations if s else []

    @staticmethod
    def calculate_composition(sequence: str) -> Dict[str, float]:
        if not sequence:
            return {"A": 0.0, "C": 0.0, "G": 0.0, "T": 0.0}
        cnt = Counter(sequence.upper())
        return {b: (cnt.get(b, 0) / len(sequence)) * 100.0 for b in "ACGT"}

    @staticmethod
    def calculate_trf_score(consensus: str, copies: int, mismatch_rate: float, length: int) -> int:
        good = length * (1.0 - mismatch_rate)
        bad = length * mismatch_rate
        return max(0, int((good * 2) - (bad * 7)))

    @staticmethod
    def calculate_trf_statistics(text_arr: np.ndarray, start: int, end: int, consensus_motif: str,
                                 copies: int, mismatch_rate: float):
        if end <= text_arr.size:
            actual = text_arr[start:end].tobytes().decode("ascii", errors="replace")
        else:
            actual = consensus_motif * int(copies)
        return ((1.0 - mismatch_rate) * 100.0, 0.0,
                MotifUtils.calculate_trf_score(consensus_motif, copies, mismatch_rate, end - start),
                MotifUtils.calculate_composition(consensus_motif),
                MotifUtils.calculate_entropy(consensus_motif), actual)

    @staticmethod
    def enumerate_motifs(k: int, alphabet: str = "ACGT") -> Iterator[str]:
        """bwt.py:1369-1381: canonical (least rotation) primitive strings of
        length k in itertools.product order.  Vectorised for k >= 1 over a
        duplicate-free alphabet: a string is its own least rotation iff no
        rotation is smaller, and primitive iff no non-trivial rotation equals
        it (motif[:p] * (k // p) == motif <=> rotation by p is the identity)."""
        a = len(alphabet)
        if k >= 1 and a >= 1 and len(set(alphabet)) == a and a ** k <= 1 << 22:
            rank = np.argsort(np.argsort([ord(c) for c in alphabet]))   # string order of each symbol
            idx = np.arange(a ** k, dtype=np.int64)
            digits = np.stack([(idx // a ** (k - 1 - j)) % a for j in range(k)], axis=1)
            w = np.array([a ** (k - 1 - j) for j in range(k)], dtype=np.int64)
            r = rank[digits]
            val = r @ w
            keep = np.ones(idx.size, dtype=bool)
            for s in range(1, k):
                rot = np.roll(r, -s, axis=1) @ w
                keep &= rot > val          # smaller rotation -> not canonical; equal -> not primitive
            chars = np.array(list(alphabet))
            for row in digits[keep]:
                yield "".join(chars[row])
            return
        for tup in product(alphabet, repeat=k):
            s = "".join(tup)
            if MotifUtils.get_canonical_motif(s) == s and MotifUtils.is_primitive_motif(s):
                yield s
