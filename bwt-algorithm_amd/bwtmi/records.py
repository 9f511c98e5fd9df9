"""Repeat records and the native job wrapper.

``TandemRepeat`` keeps the reference's field names and formatters
(bwt.py:429-641) so user code that consumed the reference's objects keeps
working; the bulk path never materialises them -- ``RepeatList`` is a lazy
view over the records held by the native job, and ``save_results`` renders
them natively (bwt.py:4141-4198).
"""
from __future__ import annotations

import ctypes as C
import os
import functools
import math
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence

import numpy as np

from . import _lib
from ._lib import Hit, Params, check, lib


@dataclass
class TandemRepeat:
    chrom: str
    start: int
    end: int
    motif: str
    copies: float
    length: int
    tier: int
    confidence: float = 1.0
    consensus_motif: Optional[str] = None
    mismatch_rate: float = 0.0
    max_mismatches_per_copy: int = 0
    n_copies_evaluated: int = 0
    strand: str = "+"
    percent_matches: float = 0.0
    percent_indels: float = 0.0
    score: int = 0
    composition: Optional[Dict[str, float]] = None
    entropy: float = 0.0
    actual_sequence: Optional[str] = None
    variations: Optional[List[str]] = None

    # formatters: same columns and number formats as bwt.py:454-513
    def _cons(self) -> str:
        return self.consensus_motif or self.motif

    def _comp(self):
        return self.composition or {"A": 25.0, "C": 25.0, "G": 25.0, "T": 25.0}

    def to_bed(self) -> str:
        return (f"{self.chrom}\t{self.start}\t{self.end}\t{self._cons()}\t{self.copies:.1f}\t"
                f"{self.tier}\t{self.mismatch_rate:.3f}\t{self.strand}")

    def to_vcf_info(self) -> str:
        return ";".join([f"MOTIF={self.motif}", f"CONS_MOTIF={self._cons()}",
                         f"COPIES={self.copies:.1f}", f"TIER={self.tier}",
                         f"CONF={self.confidence:.2f}", f"MM_RATE={self.mismatch_rate:.3f}",
                         f"MAX_MM_PER_COPY={self.max_mismatches_per_copy}",
                         f"N_COPIES_EVAL={self.n_copies_evaluated}", f"STRAND={self.strand}"])

    def to_trf_table(self) -> str:
        c, p = self._comp(), len(self._cons())
        return (f"{self.start}--{self.end}\t{p}\t{self.copies:.1f}\t{p}\t"
                f"{self.percent_matches:.0f}\t{self.percent_indels:.0f}\t{self.score}\t"
                f"{c['A']:.0f}\t{c['C']:.0f}\t{c['G']:.0f}\t{c['T']:.0f}\t{self.entropy:.2f}")

    def to_trf_dat(self) -> str:
        c, cons = self._comp(), self._cons()
        seq = self.actual_sequence or (cons * int(self.copies))
        return (f"{self.start} {self.end} {len(cons)} {self.copies:.1f} {len(cons)} "
                f"{self.percent_matches:.0f} {self.percent_indels:.0f} {self.score} "
                f"{c['A']:.0f} {c['C']:.0f} {c['G']:.0f} {c['T']:.0f} {self.entropy:.2f} {cons} {seq}")


def _composition(s: str) -> Dict[str, float]:
    return dict(_composition_of(s))     # a record's own dict (callers may change it)


@functools.lru_cache(maxsize=1 << 16)   # motifs recur across records
def _composition_of(s: str) -> Dict[str, float]:
    if not s:
        return {"A": 0.0, "C": 0.0, "G": 0.0, "T": 0.0}
    u = s.upper()
    return {b: (u.count(b) / len(s)) * 100.0 for b in "ACGT"}


@functools.lru_cache(maxsize=1 << 16)
def _entropy(s: str) -> float:
    if not s:
        return 0.0
    seen: Dict[str, int] = {}
    for ch in s:
        seen[ch] = seen.get(ch, 0) + 1
    e = 0.0
    for c in seen.values():
        p = c / len(s)
        e -= p * np.log2(p)            # MotifUtils.calculate_entropy uses np.log2 (bwt.py:730-745)
    return float(e)


# bwtmi_hit as a numpy record (same layout as the ctypes Hit)
_HIT_DTYPE = np.dtype([("start", "<i8"), ("end", "<i8"), ("unit_len", "<i4"), ("prim_len", "<i4"),
                       ("copies", "<i8")])
assert _HIT_DTYPE.itemsize == C.sizeof(Hit)


class Job:
    """Owner of one native bwtmi_job (contigs, raw hits, final records)."""

    def __init__(self, min_copies=3, max_unit_len=120, show_progress=False, tier2=True,
                 threads=0, build_index=False, sa_sample=32):
        self.params = Params(min_copies, max_unit_len, int(bool(show_progress)), int(bool(tier2)),
                             threads, int(bool(build_index)), sa_sample, 0)
        self.h = C.c_void_p()
        check(lib().bwtmi_job_create(C.byref(self.params), C.byref(self.h)))
        self.names: List[str] = []

    def __del__(self):
        h = getattr(self, "h", None)
        if h and _lib._lib is not None:
            _lib._lib.bwtmi_job_free(h)
            self.h = None

    # contigs ------------------------------------------------------------
    def add_contig(self, name: str, full: bytes, trim_left: int, trim_right: int) -> int:
        cid = C.c_int32()
        buf = C.create_string_buffer(full, len(full)) if full else None
        check(lib().bwtmi_job_add_contig(self.h, name.encode(), buf, len(full), trim_left, trim_right,
                                         C.byref(cid)))
        self.names.append(name)
        return cid.value

    def load_fasta(self, path: str, flank_trim: int, world: int = 1, rank: int = 0, comm=None,
                   dev_ctx=None) -> None:
        """load_reference (bwt.py:3713-3756), natively; with world > 1 only this
        rank's fold units get their bases (and the job is restricted to them).
        With a communicator (bwtmi.comm) no rank reads the whole file: each scans
        its 1/world, the part tables are all-gathered, each reads its own contigs.
        With a device context (whole file, or the split load) the analysed
        sequences are built on the device from the file bytes and the host copies
        are written behind the next scan (bwtmi_job_load_fasta_dev /
        _parts_dev): upload() has nothing left to do."""
        from . import profile
        with profile.stage("load", os.path.getsize(path) if os.path.exists(path) else 0):
            self._load_fasta(path, flank_trim, world, rank, comm, dev_ctx)
        if profile.active() is not None:
            profile.active().info["bases"] = int(sum(self.contig_weight(i) for i in range(self.contig_count())))

    def _load_fasta(self, path, flank_trim, world, rank, comm, dev_ctx) -> None:
        if dev_ctx is not None and world <= 1:
            check(lib().bwtmi_job_load_fasta_dev(dev_ctx, self.h, path.encode(), flank_trim))
        elif world > 1 and comm is not None:
            from . import comm as _comm
            blob, nw = C.c_void_p(), C.c_int64()
            if dev_ctx is not None:   # the part's bytes go up to the device during the exchange
                check(lib().bwtmi_job_fasta_scan_part_dev(dev_ctx, self.h, path.encode(), world, rank, C.byref(blob),
                                                          C.byref(nw)))
            else:
                check(lib().bwtmi_job_fasta_scan_part(self.h, path.encode(), world, rank, C.byref(blob),
                                                      C.byref(nw)))
            try:
                mine = np.ctypeslib.as_array(C.cast(blob, C.POINTER(C.c_int64)), shape=(nw.value,)).copy()
            finally:
                lib().bwtmi_free(blob)
            parts = np.frombuffer(b"".join(_comm.allgather_bytes(comm, mine.tobytes())), dtype=np.int64)
            if dev_ctx is not None:
                check(lib().bwtmi_job_load_fasta_parts_dev(dev_ctx, self.h, path.encode(), flank_trim, world, rank,
                                                          parts.ctypes.data_as(C.c_void_p), parts.size))
            else:
                check(lib().bwtmi_job_load_fasta_parts(self.h, path.encode(), flank_trim, world, rank,
                                                      parts.ctypes.data_as(C.c_void_p), parts.size))
        elif world > 1:
            check(lib().bwtmi_job_load_fasta_shard(self.h, path.encode(), flank_trim, world, rank))
        else:
            check(lib().bwtmi_job_load_fasta(self.h, path.encode(), flank_trim))
        if len(self.names) != self.contig_count():
            self.names = [self.contig_info(i)[0] for i in range(self.contig_count())]

    def contig_weight(self, i: int) -> int:
        """Analysed (trimmed) length of contig i, also when its bases are on another rank."""
        return lib().bwtmi_job_contig_weight(self.h, i)

    def select_shard(self, world: int, rank: int) -> List[int]:
        """Restrict the job to this rank's fold units (LPT over analysed lengths)."""
        ids = np.zeros(max(1, self.contig_count()), dtype=np.int32)
        n = C.c_int32()
        check(lib().bwtmi_job_select_shard(self.h, world, rank, ids.ctypes.data_as(C.c_void_p), C.byref(n)))
        return ids[:n.value].tolist()

    def contig_count(self) -> int:
        return lib().bwtmi_job_contig_count(self.h)

    def contig_info(self, i: int):
        fl, tl, tr = C.c_int64(), C.c_int64(), C.c_int64()
        n = lib().bwtmi_job_contig_info(self.h, i, None, 0, C.byref(fl), C.byref(tl), C.byref(tr))
        buf = C.create_string_buffer(n + 1)
        lib().bwtmi_job_contig_info(self.h, i, buf, n + 1, None, None, None)
        return buf.value.decode(errors="surrogateescape"), fl.value, tl.value, tr.value

    def contig_seq(self, i: int) -> bytes:
        _, fl, _, _ = self.contig_info(i)
        buf = C.create_string_buffer(max(fl, 1))
        check(lib().bwtmi_job_contig_seq(self.h, i, buf))
        return buf.raw[:fl]

    def device_text(self, dev_ctx, i: int) -> bytes:
        """The device copy of contig i's analysed (trimmed) sequence."""
        _, fl, tl, tr = self.contig_info(i)
        n = fl - tl - tr
        buf = C.create_string_buffer(max(n, 1))
        check(lib().bwtmi_job_device_text(dev_ctx, self.h, i, buf))
        return buf.raw[:n]

    # pipeline -----------------------------------------------------------
    def upload(self, dev_ctx) -> None:
        from . import profile
        with profile.stage("upload"):
            check(lib().bwtmi_job_upload(dev_ctx, self.h))

    def scan(self, dev_ctx) -> None:
        from . import profile
        with profile.stage("scan"):
            check(lib().bwtmi_job_scan(dev_ctx, self.h))

    def wait(self, dev_ctx) -> None:
        """Join the background FM index builds started by scan()."""
        from . import profile
        with profile.stage("index_wait"):
            check(lib().bwtmi_job_wait(dev_ctx, self.h))
        if profile.active() is not None:
            profile.active().job_split(self)

    def reset(self) -> None:
        check(lib().bwtmi_job_reset(self.h))

    def set_tier2(self, on: bool) -> None:
        self.params.tier2 = int(bool(on))
        check(lib().bwtmi_job_set_params(self.h, C.byref(self.params)))

    def set_build_index(self, on: bool) -> None:
        self.params.build_index = int(bool(on))
        check(lib().bwtmi_job_set_params(self.h, C.byref(self.params)))

    def select(self, ids) -> None:
        """Scan only these contig ids (this rank's shard); None = all."""
        if ids is None:
            check(lib().bwtmi_job_select(self.h, None, -1))
            return
        arr = np.asarray(list(ids), dtype=np.int32)
        buf = arr if arr.size else np.zeros(1, dtype=np.int32)
        check(lib().bwtmi_job_select(self.h, buf.ctypes.data_as(C.c_void_p), int(arr.size)))

    def add_hits(self, cid: int, hits: np.ndarray) -> None:
        """hits: int64[k,5] rows (start, end, unit_len, prim_len, copies)."""
        hits = np.asarray(hits, dtype=np.int64).reshape(-1, 5)
        arr = np.zeros(max(len(hits), 1), dtype=_HIT_DTYPE)
        for k, name in enumerate(_HIT_DTYPE.names):
            arr[name][:len(hits)] = hits[:, k]
        check(lib().bwtmi_job_add_hits(self.h, cid, arr.ctypes.data_as(C.c_void_p), len(hits)))

    def raw_count(self) -> int:
        return lib().bwtmi_job_raw_count(self.h)

    def postprocess(self) -> None:
        from . import profile
        with profile.stage("postprocess"):
            check(lib().bwtmi_job_postprocess(self.h))
        if profile.active() is not None:
            profile.active().info["records"] = self.count()

    def count(self) -> int:
        return lib().bwtmi_job_count(self.h)

    def render(self, fmt: str = "strfinder") -> bytes:
        p, n = C.c_void_p(), C.c_int64()
        check(lib().bwtmi_job_render(self.h, _lib.FMT[fmt], C.byref(p), C.byref(n)))
        try:
            return C.string_at(p, n.value)
        finally:
            lib().bwtmi_free(p)

    def write(self, fmt: str, path: str, background: bool = False) -> None:
        """Write the file (bwtmi_job_write).  background=True returns once the
        rows are formatted and the job's writer finishes the file behind the
        caller (bwtmi_job_write_async): write_join() waits for it and raises
        its error; the next write and the job's release join it first."""
        from . import profile
        with profile.stage("write"):
            fn = lib().bwtmi_job_write_async if background else lib().bwtmi_job_write
            check(fn(self.h, _lib.FMT[fmt], path.encode()))
        if profile.active() is not None and not background:
            profile.active().add_bytes("write", os.path.getsize(path))

    def write_join(self) -> None:
        check(lib().bwtmi_job_write_join(self.h))

    # ---- sharded output (bwtmi.dist.write_sharded)
    def unit_count(self) -> int:
        return lib().bwtmi_job_unit_count(self.h)

    def unit_rows(self) -> np.ndarray:
        out = np.zeros(self.unit_count(), dtype=np.int64)
        check(lib().bwtmi_job_unit_rows(self.h, out.ctypes.data))
        return out

    def render_units(self, fmt: str, row_base: Optional[np.ndarray] = None) -> np.ndarray:
        """Format the local fold units; returns [header bytes, bytes of unit 0, ...]."""
        out = np.zeros(self.unit_count() + 1, dtype=np.int64)
        rb = None
        if row_base is not None:
            row_base = np.ascontiguousarray(row_base, dtype=np.int64)
            rb = row_base.ctypes.data
        from . import profile
        with profile.stage("write"):
            check(lib().bwtmi_job_render_units(self.h, _lib.FMT[fmt], rb, out.ctypes.data))
        return out

    def write_units(self, path: str, offsets: np.ndarray, write_header: bool, background: bool = False) -> None:
        """pwrite the rendered units at `offsets`; background=True returns at once
        and write_join() waits for the job's writer (bwtmi_job_write_units_async)."""
        offsets = np.ascontiguousarray(offsets, dtype=np.int64)
        from . import profile
        with profile.stage("write"):
            fn = lib().bwtmi_job_write_units_async if background else lib().bwtmi_job_write_units
            check(fn(self.h, path.encode(), offsets.ctypes.data, int(write_header)))

    def export(self) -> bytes:
        p, n = C.c_void_p(), C.c_int64()
        check(lib().bwtmi_job_export(self.h, C.byref(p), C.byref(n)))
        try:
            return C.string_at(p, n.value)
        finally:
            lib().bwtmi_free(p)

    def contig_errors(self) -> Dict[int, str]:
        """{contig id: message} of the contigs whose worker failed in the last scan."""
        out = {}
        for i in range(self.contig_count()):
            n = lib().bwtmi_job_contig_error(self.h, i, None, 0)
            if n > 0:
                buf = C.create_string_buffer(n + 1)
                lib().bwtmi_job_contig_error(self.h, i, buf, n + 1)
                out[i] = buf.value.decode(errors="replace")
        return out

    def set_records(self, repeats: Sequence["TandemRepeat"], full_sequences: Dict[str, str]) -> None:
        """Replace the final records by caller-provided TandemRepeat objects
        (save_results over a plain list, bwt.py:4141-4198).  actual_sequence
        must be None or the slice full_sequence[start:end] of its contig."""
        import struct
        ids = {}
        for i, nm in enumerate(self.names):
            ids.setdefault(nm, i)
        hdr = struct.Struct("<ii8q5d5b3xii")
        if hdr.size != lib().bwtmi_wire_record_size():
            raise RuntimeError("record wire format mismatch with libbwtmi")
        parts = [struct.pack("<q", len(repeats))]
        for r in repeats:
            if r.chrom not in ids:
                raise KeyError(f"record for unknown chromosome {r.chrom!r}")
            if r.consensus_motif not in (None, r.motif):
                raise ValueError("records whose consensus_motif differs from motif are not supported")
            kind, off, ln = 0, 0, 0
            if r.actual_sequence is not None:
                full = full_sequences[r.chrom]
                if full[r.start:r.end] != r.actual_sequence:
                    raise ValueError("actual_sequence must be the slice [start:end) of the contig")
                kind, off, ln = 2, max(0, min(r.start, len(full))), len(r.actual_sequence)
            comp = r.composition
            stats_none = comp is None and r.entropy == 0.0
            kmer = comp is not None and all(v == 0 for v in comp.values()) and r.entropy == 1.5
            motif = r.motif.encode("latin-1")
            var = ";".join(r.variations).encode("latin-1") if r.variations else b""
            parts.append(hdr.pack(ids[r.chrom], int(r.tier), int(r.start), int(r.end), int(r.length),
                                  int(r.max_mismatches_per_copy), int(r.n_copies_evaluated), int(r.score), off, ln,
                                  float(r.copies), float(r.confidence), float(r.mismatch_rate),
                                  float(r.percent_matches), float(r.percent_indels), kind, ord(r.strand[:1] or "+"),
                                  0, int(kmer), int(stats_none), len(motif), len(var)))
            parts.append(motif)
            parts.append(var)
        blob = b"".join(parts)
        buf = C.create_string_buffer(blob, len(blob))
        check(lib().bwtmi_job_set_records(self.h, buf, len(blob)))

    def import_records(self, blob: bytes) -> None:
        buf = C.create_string_buffer(blob, len(blob))
        check(lib().bwtmi_job_import(self.h, buf, len(blob)))

    def stage_ms(self) -> List[float]:
        out = (C.c_double * 8)()
        check(lib().bwtmi_job_stage_ms(self.h, out))
        return list(out)

    # record view --------------------------------------------------------
    def _string(self, i: int, which: int) -> str:
        n = lib().bwtmi_job_get_string(self.h, i, which, None, 0)
        if n <= 0:
            return ""
        buf = C.create_string_buffer(n)
        lib().bwtmi_job_get_string(self.h, i, which, buf, n)
        return buf.raw[:n].decode("ascii", errors="replace")

    def records(self) -> "RepeatList":
        return RepeatList(self)


class RepeatList(Sequence):
    """Lazy sequence of TandemRepeat over a job's final records (sorted as the
    reference returns them)."""

    def __init__(self, job: Job):
        self.job = job
        n = job.count()
        self._n = n
        self._ints = np.zeros((max(n, 1), 9), dtype=np.int64)
        self._dbls = np.zeros((max(n, 1), 5), dtype=np.float64)
        if n:
            check(lib().bwtmi_job_get_records(job.h, self._ints.ctypes.data_as(C.c_void_p),
                                              self._dbls.ctypes.data_as(C.c_void_p)))
        self._cache: Dict[int, TandemRepeat] = {}
        self._cols: Dict[int, tuple] = {}

    def _str(self, i: int, which: int) -> str:
        """String `which` of record i from its column, fetched whole on first use
        (bwtmi_job_get_strings: two C calls per column, not two per record)."""
        col = self._cols.get(which)
        if col is None:
            off = np.zeros(self._n + 1, dtype=np.int64)
            tot = lib().bwtmi_job_get_strings(self.job.h, which, None, 0, off.ctypes.data_as(C.c_void_p))
            buf = C.create_string_buffer(max(int(tot), 1))
            if tot > 0:
                lib().bwtmi_job_get_strings(self.job.h, which, buf, tot, None)
            col = self._cols[which] = (buf.raw[:max(int(tot), 0)], off.tolist())
        raw, off = col
        return raw[off[i]:off[i + 1]].decode("ascii", errors="replace")

    def __len__(self):
        return self._n

    def __getitem__(self, i):
        if isinstance(i, slice):
            return [self[k] for k in range(*i.indices(self._n))]
        if i < 0:
            i += self._n
        if not 0 <= i < self._n:
            raise IndexError(i)
        r = self._cache.get(i)
        if r is None:
            s, e, ln, tier, neval, maxmm, score, flags, chrom = self._ints[i].tolist()
            copies, mm, conf, pmatch, pindel = self._dbls[i].tolist()
            motif = self._str(i, 0)
            var = self._str(i, 2)
            act = self._str(i, 3)
            if flags & 1:      # a bare consolidated Tier 3 call (bwt.py:3021-3030)
                cons, comp, ent = None, None, 0.0
            elif flags & 2:    # compound-stage k-mer piece (bwt.py:3980-3987)
                cons, comp, ent = motif, {"A": 0, "C": 0, "G": 0, "T": 0}, 1.5
            else:
                cons, comp, ent = motif, _composition(motif), _entropy(motif)
            r = TandemRepeat(chrom=self.job.names[chrom], start=s, end=e, motif=motif, copies=copies,
                             length=ln, tier=tier, confidence=conf, consensus_motif=cons,
                             mismatch_rate=mm, max_mismatches_per_copy=maxmm,
                             n_copies_evaluated=neval, strand=self._str(i, 4),
                             percent_matches=pmatch, percent_indels=pindel, score=score,
                             composition=comp, entropy=ent, actual_sequence=act if act else None,
                             variations=var.split(";") if var else None)
            self._cache[i] = r
        return r
