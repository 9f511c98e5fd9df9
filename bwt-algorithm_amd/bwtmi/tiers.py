"""Detector classes of the reference (bwt.py:1387-3036).

Tier2LCPFinder.find_long_unit_repeats_strict -- the detector that decides the
CLI's repeat.tab -- runs on the device (libbwtmi strict scan); the LCP array
comes from the device index.  The library-only finders that the CLI never
calls run over the device index
as well (library.hip).
"""
from __future__ import annotations

import ctypes as C
from typing import List, Optional, Set, Tuple

import numpy as np

from . import _lib
from ._lib import Hit, check, lib
from .motif import MotifUtils
from .records import TandemRepeat


def strict_scan_hits(text_arr: np.ndarray, min_unit: int, max_unit: int, min_copies: int,
                     device: Optional[int] = None, max_mismatch: int = 0) -> np.ndarray:
    """Device strict scan -> int64[k, 5] rows (start, end, unit_len, prim_len, copies);
    max_mismatch > 0 takes the Hamming-tolerant adjacency (bwt.py:1929-1944)."""
    t = np.ascontiguousarray(text_arr, dtype=np.uint8)
    buf = t if t.size else np.zeros(1, dtype=np.uint8)
    out = C.POINTER(Hit)()
    n = C.c_int64()
    check(lib().bwtmi_strict_scan(_lib.ctx(device), buf.ctypes.data_as(C.c_void_p), t.size, min_unit,
                                  max_unit, max_mismatch, min_copies, C.byref(out), C.byref(n)))
    try:
        if n.value == 0:
            return np.zeros((0, 5), dtype=np.int64)
        raw = np.ctypeslib.as_array(C.cast(out, C.POINTER(C.c_int64)), shape=(n.value * 4,))
        rec = raw.reshape(n.value, 4).copy()
    finally:
        lib().bwtmi_free(out)
    res = np.empty((n.value, 5), dtype=np.int64)
    res[:, 0] = rec[:, 0]
    res[:, 1] = rec[:, 1]
    res[:, 2] = rec[:, 2] & 0xFFFFFFFF
    res[:, 3] = rec[:, 2] >> 32
    res[:, 4] = rec[:, 3]
    return res


class Tier1STRFinder:
    """bwt.py:1387-1862 -- library-only sliding-window finder (never reached by
    the CLI: `--tier1` disables Tier 2 and the worker ignores Tier 1)."""

    def __init__(self, text_arr: np.ndarray, max_motif_length: int = 9, show_progress: bool = False):
        self.text_arr = text_arr
        self.max_motif_length = max_motif_length
        self.min_copies = 3
        self.min_array_length = 6
        self.min_entropy = 1.0
        self.show_progress = show_progress

    def find_strs(self, chromosome: str) -> List[TandemRepeat]:
        """bwt.py:1426-1538: perfect 1-9 bp arrays, longest unit first, with the
        reference's seen-mask and position step; stop positions are decided on
        the device per unit length (library.hip), the walk itself on the host."""
        from .records import Job
        t = np.ascontiguousarray(self.text_arr, dtype=np.uint8)
        job = Job()
        job.add_contig(chromosome, t.tobytes(), 0, 0)
        check(lib().bwtmi_job_tier1(_lib.ctx(), job.h, 0, int(self.max_motif_length)))
        return list(job.records())


class Tier2LCPFinder:
    def __init__(self, bwt_core, min_period: int = 1, max_period: int = 1000, max_short_motif: int = 9,
                 allow_mismatches: bool = True, show_progress: bool = False):
        self.bwt = bwt_core
        self.min_period = min_period
        self.max_period = max_period
        self.max_short_motif = max_short_motif
        self.min_copies = 3
        self.min_array_length = 6
        self.min_entropy = 1.0
        self.allow_mismatches = allow_mismatches
        self.show_progress = show_progress
        self.period_step = 1

    def find_long_unit_repeats_strict(self, chromosome: str, min_unit_len: int = 20,
                                      max_unit_len: int = 120, max_mismatch: int = 2,
                                      min_copies: int = 3) -> List[TandemRepeat]:
        """bwt.py:1891-2001 on the device (records built as bwt.py:1952-1993)."""
        t = self.bwt.text_arr
        hits = strict_scan_hits(t, min_unit_len, max_unit_len, min_copies, max_mismatch=max_mismatch)
        out = []
        for s, e, L, p, c in hits.tolist():
            motif = bytes(t[s:s + p]).decode("ascii", errors="replace")
            pm, pi, sc, comp, ent, act = MotifUtils.calculate_trf_statistics(t, s, e, motif, c, 0.0)
            out.append(TandemRepeat(
                chrom=chromosome, start=s, end=e, motif=motif, copies=float(c), length=e - s, tier=2,
                confidence=0.95, consensus_motif=motif, mismatch_rate=0.0,
                max_mismatches_per_copy=0 if pm >= 99.9 else max_mismatch, n_copies_evaluated=c,
                strand="+", percent_matches=pm, percent_indels=pi, score=sc, composition=comp,
                entropy=ent, actual_sequence=act, variations=None))
        return out

    def _compute_lcp_array(self) -> np.ndarray:
        """bwt.py:2108-2116 (Kasai) -- device LCP."""
        if self.bwt.n == 0:
            return np.zeros(0, dtype=np.int32)
        return self.bwt.lcp_array()

    def _params(self) -> "_lib.LibParams":
        return _lib.LibParams(self.min_period, self.max_period, self.max_short_motif, self.min_copies,
                              self.min_array_length, int(bool(self.allow_mismatches)), float(self.min_entropy))

    def find_short_imperfect_repeats(self, chromosome: str, tier1_seen: Set[Tuple[int, int]]) -> List[TandemRepeat]:
        """bwt.py:2027-2095: k-mer-table / FM seeds for every canonical motif of
        length min_period..9, Hamming seed-and-extend with majority-vote
        consensus (device extension table, library.hip), records as bwt.py:2653-2691."""
        from .records import Job
        t = np.ascontiguousarray(self.bwt.text_arr, dtype=np.uint8)
        if t.size > 1_000_000:                                   # bwt.py:2048-2051
            if self.show_progress:
                print(f"  [{chromosome}] Tier 2 short imperfect repeats: SKIPPED (>{t.size:,} bp, too expensive)")
            return []
        job = Job()
        job.add_contig(chromosome, t.tobytes(), 0, 0)
        seen = np.array(sorted(tier1_seen or ()), dtype=np.int64).reshape(-1)
        buf = seen if seen.size else np.zeros(2, dtype=np.int64)
        p = self._params()
        check(lib().bwtmi_index_short_imperfect(self.bwt._ctx, self.bwt._h, C.byref(p), buf.ctypes.data,
                                                seen.size // 2, job.h, 0))
        return list(job.records())

    def _detect_lcp_plateaus(self, lcp_array: np.ndarray, chromosome: str) -> List[TandemRepeat]:
        """bwt.py:2118-2145 with _analyze_sa_interval_for_tandems (2500-2549) on the
        device.  The LCP used is this finder's own Kasai array (what
        _compute_lcp_array() returns), recomputed on the device."""
        out = C.c_void_p()
        n = C.c_int64()
        p = self._params()
        check(lib().bwtmi_index_lcp_plateaus(self.bwt._ctx, self.bwt._h, C.byref(p), C.byref(out), C.byref(n)))
        try:
            trip = (np.ctypeslib.as_array(C.cast(out, C.POINTER(C.c_int64)), shape=(n.value * 3,)).copy()
                    if n.value else np.zeros(0, dtype=np.int64))
        finally:
            lib().bwtmi_free(out)
        t = self.bwt.text_arr
        res = []
        for s, c, per in trip.reshape(-1, 3).tolist():
            res.append(TandemRepeat(chrom=chromosome, start=s, end=s + c * per,
                                    motif=bytes(t[s:s + per]).decode("ascii"), copies=c, length=c * per,
                                    tier=2, confidence=0.9))
        return res

    def find_long_repeats(self, chromosome: str, tier1_seen: Optional[Set[Tuple[int, int]]] = None):
        """bwt.py:2097-2106 -> _find_repeats_simple (2177-2390): one walk per
        period over the positions, first extensions (_extend_with_mismatches,
        2392-2498) evaluated on the device in look-ahead batches (library.hip).
        The reference's 30 s wall-clock stop (2238-2257) is not reproduced."""
        return self._find_repeats_simple(chromosome, tier1_seen or set())

    def _find_repeats_simple(self, chromosome: str, tier1_seen: Set[Tuple[int, int]]) -> List[TandemRepeat]:
        from .records import Job
        t = np.ascontiguousarray(self.bwt.text_arr, dtype=np.uint8)
        job = Job()
        job.add_contig(chromosome, t.tobytes(), 0, 0)
        seen = np.array(sorted(tier1_seen or ()), dtype=np.int64).reshape(-1)
        buf = seen if seen.size else np.zeros(2, dtype=np.int64)
        p = self._params()
        check(lib().bwtmi_index_long_repeats(self.bwt._ctx, self.bwt._h, C.byref(p), buf.ctypes.data,
                                             seen.size // 2, job.h, 0))
        return list(job.records())


def pack_reads(long_reads) -> Tuple[np.ndarray, np.ndarray]:
    """Reads (str or bytes) back to back + int64 offsets[n + 1]."""
    bs = [r if isinstance(r, (bytes, bytearray)) else r.encode("latin-1", errors="replace") for r in long_reads]
    off = np.zeros(len(bs) + 1, dtype=np.int64)
    if bs:
        off[1:] = np.cumsum([len(b) for b in bs])
    blob = np.frombuffer(b"".join(bs), dtype=np.uint8) if off[-1] else np.zeros(1, dtype=np.uint8)
    return np.ascontiguousarray(blob), off


class Tier3LongReadFinder:
    """bwt.py:2828-3036 -- long-read anchoring.  The window periodicity scan
    (500-byte windows every 100 bytes, periods 10..165) and the anchor lookups
    (backward search + SA of the 50-byte anchors) run on the device over the
    core's index; records are built and consolidated natively (library.hip)."""

    def __init__(self, bwt_core, show_progress: bool = False):
        self.bwt = bwt_core
        self.min_read_length = 1000  # bwt.py:2833
        self.min_span_length = 100   # bwt.py:2834 (unused by the reference too)
        self.show_progress = show_progress

    def _run(self, long_reads, job, contig_id: int, as_input: bool) -> None:
        blob, off = pack_reads(long_reads)
        check(lib().bwtmi_index_tier3(self.bwt._ctx, self.bwt._h, blob.ctypes.data_as(C.c_void_p),
                                      off.ctypes.data_as(C.c_void_p), len(off) - 1, job.h, contig_id,
                                      int(as_input)))

    def find_very_long_repeats(self, long_reads: List[str], chromosome: str) -> List[TandemRepeat]:
        from .records import Job
        t = np.ascontiguousarray(self.bwt.text_arr, dtype=np.uint8)
        job = Job()
        job.add_contig(chromosome, t.tobytes(), 0, 0)
        self._run(long_reads, job, 0, False)
        return list(job.records())
