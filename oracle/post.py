"""Pure-Python restatement of the reference's record construction and the
sequential repeat post-processing -- TEST INFRASTRUCTURE (see oracle/__init__).

Reference: /root/reference/bwt.py (wyim-pgl/bwt-algorithm @ 2025-11-14).
Each function names the lines it restates.  Used by tests (as the checker of
the product's C++ post-processing) and by tests/golden/make_goldens.py (the
"hybrid" oracle that produces full-size goldens).
"""
from __future__ import annotations

import bisect
import math
import re
from collections import Counter
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

# --------------------------------------------------------------------------
# small motif helpers (MotifUtils, bwt.py:675-1381)
# --------------------------------------------------------------------------
_RC = {"A": "T", "T": "A", "C": "G", "G": "C", "N": "N"}


def natural_key(name):                       # _natural_sort_key bwt.py:22-36
    if name is None:
        return ()
    out = []
    for part in re.split(r"(\d+)", str(name)):
        if not part:
            continue
        out.append((0, int(part)) if part.isdigit() else (1, part.lower()))
    return tuple(out)


def revcomp(s: str) -> str:                   # bwt.py:688-691
    return "".join(_RC.get(c, c) for c in reversed(s))


def min_rotation(s: str) -> str:              # bwt.py:679-685
    return min(s[i:] + s[:i] for i in range(len(s))) if s else s


def canonical_stranded(s: str) -> Tuple[str, str]:   # bwt.py:694-716
    if not s:
        return s, "+"
    f = min_rotation(s)
    r = min_rotation(revcomp(s))
    return (f, "+") if f <= r else (r, "-")


def smallest_period(s: str) -> int:           # bwt.py:1125-1133
    n = len(s)
    for p in range(1, n + 1):
        if n % p == 0 and s == s[:p] * (n // p):
            return p
    return n if n else 0


def entropy(s: str) -> float:                 # bwt.py:730-745
    if not s:
        return 0.0
    n = len(s)
    e = 0.0
    for c in Counter(s).values():
        p = c / n
        e -= p * np.log2(p)
    return e


def composition(s: str) -> Dict[str, float]:  # bwt.py:1290-1310
    if not s:
        return {"A": 0.0, "C": 0.0, "G": 0.0, "T": 0.0}
    cnt = Counter(s.upper())
    t = len(s)
    return {b: (cnt.get(b, 0) / t) * 100.0 for b in "ACGT"}


def trf_score(length: int, mm: float) -> int:   # bwt.py:1313-1333
    matches = length * (1.0 - mm)
    mism = length * mm
    return max(0, int((matches * 2) - (mism * 7)))


# --------------------------------------------------------------------------
# record
# --------------------------------------------------------------------------
class Rec:
    """Field-for-field stand-in for TandemRepeat (bwt.py:429-452)."""
    __slots__ = ("chrom", "start", "end", "motif", "copies", "length", "tier", "confidence",
                 "consensus_motif", "mismatch_rate", "max_mismatches_per_copy",
                 "n_copies_evaluated", "strand", "percent_matches", "percent_indels", "score",
                 "composition", "entropy", "actual_sequence", "variations", "is_compound",
                 "compound_partner")

    def __init__(self, **kw):
        self.consensus_motif = None
        self.confidence = 1.0
        self.mismatch_rate = 0.0
        self.max_mismatches_per_copy = 0
        self.n_copies_evaluated = 0
        self.strand = "+"
        self.percent_matches = 0.0
        self.percent_indels = 0.0
        self.score = 0
        self.composition = None
        self.entropy = 0.0
        self.actual_sequence = None
        self.variations = None
        self.is_compound = False
        self.compound_partner = None
        for k, v in kw.items():
            setattr(self, k, v)

    @property
    def cons(self) -> str:
        return self.consensus_motif or self.motif

    def key(self):
        return (natural_key(self.chrom), self.start, self.end)


def strict_record(chrom: str, text: bytes, start: int, end: int, motif: str, count: int) -> Rec:
    """Record built per strict hit: bwt.py:1952-1993 with
    calculate_trf_statistics(text, i, end, motif, count, 0.0) (1336-1366)."""
    length = end - start
    actual = text[start:end].decode("ascii", errors="replace")
    pm = (1.0 - 0.0) * 100.0
    return Rec(chrom=chrom, start=start, end=end, motif=motif, copies=float(count),
               length=length, tier=2, confidence=0.95, consensus_motif=motif,
               mismatch_rate=0.0, max_mismatches_per_copy=0 if pm >= 99.9 else 0,
               n_copies_evaluated=count, strand="+", percent_matches=pm, percent_indels=0.0,
               score=trf_score(length, 0.0), composition=composition(motif),
               entropy=entropy(motif), actual_sequence=actual, variations=None)


def worker_records(chrom: str, seq: str, hits: np.ndarray) -> List[Rec]:
    """_process_chromosome_worker (bwt.py:3040-3135) given raw strict hits
    rows (start, end, unit_len, prim_len, copies)."""
    text = seq.encode("utf-8")
    out = []
    for s, e, L, p, c in hits.tolist():
        motif = text[s:s + p].decode("ascii", errors="replace")
        r = strict_record(chrom, text, s, e, motif, c)
        m = r.cons
        if len(m) < 5 and r.copies < 30 and (r.mismatch_rate > 0 or r.max_mismatches_per_copy > 0):
            continue                                   # Rule 1, bwt.py:3118-3130
        out.append(r)
    return out


# --------------------------------------------------------------------------
# banded alignment (MotifUtils._align_unit_to_window / align_repeat_region)
# --------------------------------------------------------------------------
def align_unit(motif: str, window: str, max_indel: int, tol: int):
    """bwt.py:829-983.  Returns (consumed, ops, observed, n_sub, n_ins, n_del) or None."""
    m, n = len(motif), len(window)
    if m == 0 or n == 0:
        return None
    max_indel = max(0, max_indel)
    tol = max(0, tol)
    lo, hi = max(0, m - max_indel), min(n, m + max_indel)
    if lo > hi:
        return None
    INF = m + n + 10
    dp = [[INF] * (n + 1) for _ in range(m + 1)]
    pt = [[""] * (n + 1) for _ in range(m + 1)]
    dp[0][0] = 0
    for j in range(1, n + 1):
        dp[0][j] = j
        pt[0][j] = "I"
    for i in range(1, m + 1):
        dp[i][0] = i
        pt[i][0] = "D"
    band = max_indel + 2
    for i in range(1, m + 1):
        mi = motif[i - 1]
        row, prev = dp[i], dp[i - 1]
        for j in range(max(1, i - band), min(n, i + band) + 1):
            eq = mi == window[j - 1]
            best = prev[j - 1] + (0 if eq else 1)
            op = "M" if eq else "S"
            if prev[j] + 1 < best:
                best, op = prev[j] + 1, "D"
            if row[j - 1] + 1 < best:
                best, op = row[j - 1] + 1, "I"
            row[j] = best
            pt[i][j] = op
    bj, bc = -1, INF
    for j in range(lo, hi + 1):
        if dp[m][j] < bc:
            bc, bj = dp[m][j], j
    if bj <= 0 or bc >= INF:
        return None
    cols = []
    i, j = m, bj
    while i > 0 or j > 0:
        op = pt[i][j]
        if op in ("M", "S"):
            cols.append((motif[i - 1], window[j - 1])); i -= 1; j -= 1
        elif op == "D":
            cols.append((motif[i - 1], "-")); i -= 1
        elif op == "I":
            cols.append(("-", window[j - 1])); j -= 1
        else:
            break
    cols.reverse()
    ops, obs = [], []
    n_sub = n_ins = n_del = 0
    ref = 0
    ins_buf: List[str] = []
    ins_at = 0
    del_len = 0
    del_at = 0
    for r, q in cols:
        if r == "-":
            if not ins_buf:
                ins_at = ref
            ins_buf.append(q)
            continue
        if ins_buf:
            s = "".join(ins_buf)
            ops.append(("ins", ins_at, s)); n_ins += len(s); ins_buf = []; ins_at = 0
        ref += 1
        if q == "-":
            if del_len == 0:
                del_at = ref
            del_len += 1
            continue
        if del_len:
            ops.append(("del", del_at, del_len)); n_del += del_len; del_len = 0
        obs.append((ref - 1, q))
        if r != q:
            ops.append(("sub", ref, r, q)); n_sub += 1
    if ins_buf:
        s = "".join(ins_buf)
        ops.append(("ins", ins_at, s)); n_ins += len(s)
    if del_len:
        ops.append(("del", del_at, del_len)); n_del += del_len
    if n_sub > tol or n_ins > max_indel or n_del > max_indel:
        return None
    return bj, ops, obs, n_sub, n_ins, n_del


def _consensus(counts: List[Counter], fallback: str) -> str:   # bwt.py:986-995
    out = []
    for i, c in enumerate(counts):
        if c:
            out.append(c.most_common(1)[0][0])
        else:
            out.append(fallback[i] if i < len(fallback) else "N")
    return "".join(out)


def align_region(seq: str, start: int, end: int, template: str, frac: float = 0.1,
                 max_indel: Optional[int] = None, min_copies: int = 3):
    """bwt.py:998-1102.  Returns dict summary or None."""
    if not template or not seq:
        return None
    L = len(seq)
    start = max(0, start)
    end = min(L, end if end > start else L)
    m = len(template)
    tol = max(1, int(math.floor(m * frac)))
    max_indel = max(1, min(10, m // 2 if m >= 4 else 1)) if max_indel is None else max(0, max_indel)
    counts = [Counter() for _ in range(m)]
    copies, ops_by_copy, errs = 0, [], []
    tot_ins = tot_del = 0
    cur = template
    pos = start
    limit = min(L, max(end, start + m * min_copies) + max(m * 3, max_indel * 4))
    while pos < limit:
        win = seq[pos:min(L, pos + m + max_indel)]
        if len(win) < m - max_indel:
            break
        res = align_unit(cur, win, max_indel, tol)
        if res is None or res[0] == 0:
            break
        consumed, ops, obs, ns, ni, nd = res
        copies += 1
        ops_by_copy.append(ops)
        errs.append(ns + ni + nd)
        tot_ins += ni
        tot_del += nd
        for idx, b in obs:
            if 0 <= idx < m:
                counts[idx][b] += 1
        pos += consumed
        cur = _consensus(counts, cur)
    if copies < min_copies:
        return None
    consumed_len = pos - start
    if consumed_len <= 0:
        return None
    cons = _consensus(counts, cur)
    denom = copies * m
    var = []
    for k, ops in enumerate(ops_by_copy, 1):
        for op in ops:
            if op[0] == "sub":
                var.append(f"{k}:{op[1]}:{op[2]}>{op[3]}")
            elif op[0] == "ins":
                if op[2]:
                    var.append(f"{k}:{op[1]}:ins({op[2]})")
            elif op[0] == "del":
                if op[2] > 0:
                    var.append(f"{k}:{op[1]}:del({op[2]})")
    return dict(consensus=cons, motif_len=m, copies=copies, consumed=consumed_len,
                mismatch_rate=(sum(errs) / denom) if denom > 0 else 0.0,
                max_errors=max(errs) if errs else 0, variations=var,
                tot_ins=tot_ins, tot_del=tot_del)


# --------------------------------------------------------------------------
# the post-processing pipeline (TandemRepeatFinder, bwt.py:3144-3954)
# --------------------------------------------------------------------------
class Pipeline:
    def __init__(self, sequences: Dict[str, str], full_sequences: Dict[str, str],
                 trim_offsets: Dict[str, int], min_copies: int = 3):
        self.sequences = sequences
        self.full = full_sequences
        self.offsets = trim_offsets
        self.min_copies = min_copies

    # bwt.py:3515-3614
    def recompute(self, chrom: str, start: int, end: int, motif_len: int, tier: int) -> Rec:
        seq = self.sequences.get(chrom)
        if seq is None:
            raise ValueError(chrom)
        L = len(seq)
        m = max(1, motif_len)
        start = max(0, int(start))
        end = min(L, int(end)) if end > 0 else L
        if end <= start:
            end = min(L, start + m)
        tmpl = seq[start:start + m]
        if not tmpl:
            a = max(0, start - m)
            tmpl = seq[a:a + m]
        if not tmpl:
            tmpl = "N" * m
        s = align_region(seq, start, end, tmpl, 0.1, None, max(1, self.min_copies))
        if s is None:
            s = align_region(seq, start, end, tmpl, 0.1, None, 1)
        if s is None:
            consumed = min(L - start, max(m, end - start))
            actual = seq[start:start + consumed]
            cint = max(1, consumed // m)
            cons = tmpl if tmpl else (actual[:m] or "N")
            mm, maxe, pind, var = 0.0, 0, 0.0, None
        else:
            actual = seq[start:start + s["consumed"]]
            cint = s["copies"]
            cons = s["consensus"] or tmpl
            mm = s["mismatch_rate"]
            tb = s["copies"] * s["motif_len"]
            pind = (((s["tot_ins"] + s["tot_del"]) / tb) if tb > 0 else 0.0) * 100.0
            maxe = s["max_errors"]
            var = s["variations"] if s["variations"] else None
        tl = len(actual)
        mle = len(cons) if cons else m
        cf = float(cint)
        if tl > 0 and mle > 0:
            fr = tl / mle
            cf = float(round(fr)) if abs(fr - round(fr)) < 1e-6 else fr
        return Rec(chrom=chrom, start=start, end=start + tl, motif=cons, copies=cf, length=tl,
                   tier=tier, confidence=max(0.3, 1.0 - mm), consensus_motif=cons,
                   mismatch_rate=mm, max_mismatches_per_copy=maxe,
                   n_copies_evaluated=max(1, cint), strand=canonical_stranded(cons)[1],
                   percent_matches=max(0.0, 100.0 - mm * 100.0), percent_indels=pind,
                   score=trf_score(tl, mm), composition=composition(cons),
                   entropy=entropy(cons), actual_sequence=actual, variations=var)

    # bwt.py:3402-3497, restated class by class: a repeat is only ever tested
    # against kept spans with a strictly longer motif, and the sort key puts
    # all longer motifs of its class (and all of the perfect class) ahead of
    # it, so every (class, motif length) group can be screened against the
    # spans kept so far and then appended as a whole.
    def suppress_nested(self, recs: List[Rec], thr: float = 0.5) -> List[Rec]:
        by: Dict[str, List[Rec]] = {}
        for r in recs:
            by.setdefault(r.chrom, []).append(r)
        kept_all: List[Rec] = []
        B = 4096
        for chrom, rs in by.items():
            order = sorted(rs, key=lambda r: (r.mismatch_rate > 0, -len(r.motif)))
            buckets: Dict[int, List[Tuple[int, int, int]]] = {}
            kept: List[Rec] = []
            g = 0
            while g < len(order):
                h = g
                cls = (order[g].mismatch_rate > 0, len(order[g].motif))
                while h < len(order) and (order[h].mismatch_rate > 0, len(order[h].motif)) == cls:
                    h += 1
                survivors = []
                for r in order[g:h]:
                    a, b, m = r.start, r.end, len(r.motif)
                    rl = b - a
                    nested = False
                    seen = set()
                    for bk in range(a // B, (max(b, a + 1) - 1) // B + 1):
                        for sp in buckets.get(bk, ()):
                            if sp in seen:
                                continue
                            seen.add(sp)
                            s, e, M = sp
                            if M <= m:
                                continue
                            ov = max(0, min(b, e) - max(a, s))
                            if ov == 0:
                                continue
                            ratio = M / m
                            if m == 1 and M > 1 and ov / rl >= 0.8:
                                nested = True
                                break
                            t = 0.1 if ratio >= 10 else (0.3 if ratio >= 5 else thr)
                            if ov / rl >= t:
                                nested = True
                                break
                        if nested:
                            break
                    if not nested:
                        survivors.append(r)
                for r in survivors:
                    kept.append(r)
                    sp = (r.start, r.end, len(r.motif))
                    for bk in range(r.start // B, (max(r.end, r.start + 1) - 1) // B + 1):
                        buckets.setdefault(bk, []).append(sp)
                g = h
            kept_all.extend(kept)      # survivors appended in the reference's sorted order
        kept_all.sort(key=Rec.key)
        return kept_all

    # bwt.py:3189-3220
    def dedup(self, recs: List[Rec]) -> List[Rec]:
        d: Dict[tuple, Rec] = {}
        for r in recs:
            k = (r.chrom, r.start, r.end, r.motif)
            ex = d.get(k)
            if ex is None:
                d[k] = r
            elif r.confidence > ex.confidence:
                d[k] = r
            elif r.confidence == ex.confidence:
                if r.mismatch_rate < ex.mismatch_rate:
                    d[k] = r
                elif r.mismatch_rate == ex.mismatch_rate and r.tier < ex.tier:
                    d[k] = r
        out = list(d.values())
        out.sort(key=Rec.key)
        return out

    # bwt.py:3240-3281
    def should_merge(self, r1: Rec, r2: Rec) -> bool:
        if r1.chrom != r2.chrom:
            return False
        m1, m2 = r1.cons, r2.cons
        if not m1 or not m2:
            return False
        if canonical_stranded(m1)[0] != canonical_stranded(m2)[0]:
            return False
        ml = min(len(m1), len(m2))
        if max(0, r2.start - r1.end) > ml + 1:
            return False
        try:
            mg = self.recompute(r1.chrom, min(r1.start, r2.start), max(r1.end, r2.end),
                                max(1, ml), min(r1.tier, r2.tier))
        except ValueError:
            return False
        if mg.copies < self.min_copies:
            return False
        return mg.mismatch_rate <= max(r1.mismatch_rate, r2.mismatch_rate, 0.01) + 0.2

    # bwt.py:3222-3238, 3283-3289
    def merge_adjacent(self, recs: List[Rec]) -> List[Rec]:
        if not recs:
            return []
        out = []
        cur = recs[0]
        for nx in recs[1:]:
            if self.should_merge(cur, nx):
                cur = self.recompute(cur.chrom, min(cur.start, nx.start), max(cur.end, nx.end),
                                     len(cur.cons), min(cur.tier, nx.tier))
            else:
                out.append(cur)
                cur = nx
        out.append(cur)
        return out

    # bwt.py:3291-3314
    def refine(self, recs: List[Rec]) -> List[Rec]:
        out = []
        for r in recs:
            if r.mismatch_rate == 0.0:
                out.append(r)
                continue
            m = len(r.cons)
            if m <= 0:
                m = max(1, r.length // max(1, int(round(r.copies)) or 1))
            out.append(self.recompute(r.chrom, r.start, r.end, m, r.tier))
        out.sort(key=Rec.key)
        return out

    # bwt.py:3316-3325
    def restore(self, recs: List[Rec]) -> None:
        for r in recs:
            off = self.offsets.get(r.chrom, 0)
            r.start += off
            r.end += off
            r.length = r.end - r.start
            fs = self.full.get(r.chrom)
            if fs:
                r.actual_sequence = fs[r.start:r.end]

    # bwt.py:3327-3354
    @staticmethod
    def should_collapse(r1: Rec, r2: Rec) -> bool:
        if r1.chrom != r2.chrom:
            return False
        ov = min(r1.end, r2.end) - max(r1.start, r2.start)
        if ov <= 0:
            return False
        sh = min(r1.length, r2.length)
        if sh <= 0 or ov / sh < 0.8:
            return False
        if canonical_stranded(r1.motif)[0] == canonical_stranded(r2.motif)[0]:
            return True
        if (len(r1.motif) == 1 or len(r2.motif) == 1) and ov / sh >= 0.95:
            return True
        if len(r1.motif) == len(r2.motif) and ov / sh >= 0.9:
            return abs(r1.mismatch_rate - r2.mismatch_rate) >= 0.2
        return False

    # bwt.py:3356-3400
    @staticmethod
    def prefer(r1: Rec, r2: Rec) -> Rec:
        m1, m2 = r1.cons, r2.cons
        l1, l2 = len(m1), len(m2)
        if l1 != l2:
            if l1 == 1 and l2 > 1:
                return r2
            if l2 == 1 and l1 > 1:
                return r1
            sh, lo = (m1, m2) if l1 < l2 else (m2, m1)
            if len(lo) % len(sh) == 0 and sh * (len(lo) // len(sh)) == lo:
                return r1 if l1 < l2 else r2
            return r1 if l1 > l2 else r2
        if r1.mismatch_rate != r2.mismatch_rate:
            return r1 if r1.mismatch_rate < r2.mismatch_rate else r2
        if r1.confidence != r2.confidence:
            return r1 if r1.confidence > r2.confidence else r2
        if r1.length != r2.length:
            return r1 if r1.length >= r2.length else r2
        return r1

    # bwt.py:3499-3513
    def collapse(self, recs: List[Rec]) -> List[Rec]:
        out: List[Rec] = []
        for r in sorted(recs, key=Rec.key):
            if out and self.should_collapse(out[-1], r):
                out[-1] = self.prefer(out[-1], r)
            else:
                out.append(r)
        return out

    # bwt.py:3926-3944
    def run(self, raw: List[Rec]) -> List[Rec]:
        recs = self.suppress_nested(raw, 0.5)
        recs = self.dedup(recs)
        recs = self.merge_adjacent(recs)
        recs = self.refine(recs)
        self.restore(recs)
        recs = self.collapse(recs)
        recs = [r for r in recs if r.copies >= self.min_copies and r.length >= 6]
        recs.sort(key=Rec.key)
        return recs

    # ---------------------------------------------------------------- output
    def _kmer_scan(self, chrom: str, start: int, end: int, k: int = 3) -> List[Rec]:
        """_simple_kmer_scan (bwt.py:3956-3993), full sequence."""
        seq = self.full.get(chrom, "")
        if not seq or start >= end or start < 0 or end > len(seq):
            return []
        reg = seq[start:end]
        out = []
        i = 0
        while i < len(reg) - k:
            mo = reg[i:i + k]
            c = 1
            j = i + k
            while j + k <= len(reg) and reg[j:j + k] == mo:
                c += 1
                j += k
            if c >= 5:
                out.append(Rec(chrom=chrom, start=start + i, end=start + j, motif=mo,
                               copies=float(c), length=j - i, tier=1, confidence=1.0,
                               consensus_motif=mo, n_copies_evaluated=c, percent_matches=100.0,
                               score=100.0, composition={"A": 0, "C": 0, "G": 0, "T": 0},
                               entropy=1.5, actual_sequence=reg[i:j]))
                i = j
            else:
                i += 1
        return out

    def compounds(self, recs: List[Rec]) -> List[Rec]:
        """_detect_compound_repeats (bwt.py:3995-4139)."""
        if not recs:
            return []
        by: Dict[str, List[Rec]] = {}
        for r in recs:
            by.setdefault(r.chrom, []).append(r)
        for chrom in by:
            seq = self.full.get(chrom, "")
            if not seq:
                continue
            for r in list(by[chrom]):
                if r.motif and len(r.motif) == 3:
                    a, b = r.end, min(len(seq), r.end + 50)
                    if a < b:
                        for kr in self._kmer_scan(chrom, a, b, 3):
                            if kr.motif != r.motif:
                                by[chrom].append(kr)
        res: List[Rec] = []
        for chrom, rs in by.items():
            rs.sort(key=lambda r: r.start)
            longs = [(r.start, r.end, len(r.motif)) for r in rs if len(r.motif) > 10]
            i = 0
            while i < len(rs):
                cur = rs[i]
                if len(cur.motif) == 3 and cur.copies >= 10:
                    seq = self.sequences.get(cur.chrom, "")
                    if seq:
                        rsq = seq[cur.start:cur.end]
                        k = len(cur.motif)
                        for sp in range(k, len(rsq) - k, k):
                            m1 = rsq[:k]
                            m2 = rsq[sp:sp + k]
                            if m1 == m2:
                                continue
                            c1 = 0
                            for j in range(0, sp, k):
                                if rsq[j:j + k] == m1:
                                    c1 += 1
                                else:
                                    break
                            c2 = 0
                            for j in range(sp, len(rsq), k):
                                if rsq[j:j + k] == m2:
                                    c2 += 1
                                else:
                                    break
                            if c1 >= 5 and c2 >= 5 and (c1 * len(m1) + c2 * len(m2)) >= len(rsq) * 0.9:
                                e1 = cur.start + c1 * len(m1)
                                r1 = Rec(chrom=cur.chrom, start=cur.start, end=e1, motif=m1,
                                         copies=float(c1), length=c1 * len(m1), tier=cur.tier,
                                         confidence=1.0, consensus_motif=m1, n_copies_evaluated=c1,
                                         percent_matches=100.0, score=100.0,
                                         composition={"A": 0, "C": 0, "G": 0, "T": 0}, entropy=1.5,
                                         actual_sequence=rsq[:c1 * len(m1)])
                                r2 = Rec(chrom=cur.chrom, start=e1, end=e1 + c2 * len(m2), motif=m2,
                                         copies=float(c2), length=c2 * len(m2), tier=cur.tier,
                                         confidence=1.0, consensus_motif=m2, n_copies_evaluated=c2,
                                         percent_matches=100.0, score=100.0,
                                         composition={"A": 0, "C": 0, "G": 0, "T": 0}, entropy=1.5,
                                         actual_sequence=rsq[c1 * len(m1):c1 * len(m1) + c2 * len(m2)])
                                r1.is_compound = True
                                r1.compound_partner = r2
                                res.append(r1)
                                i += 1
                if i + 1 < len(rs):
                    nx = rs[i + 1]
                    gap = nx.start - cur.end
                    if (gap <= 5 and len(cur.motif) <= 4 and len(nx.motif) <= 4 and
                            cur.motif != nx.motif and cur.copies >= 5 and nx.copies >= 5):
                        cs, ce = cur.start, nx.end
                        covered = False
                        for ls, le, _ in longs:
                            ov = max(0, min(ce, le) - max(cs, ls))
                            if ov / (ce - cs) >= 0.8:
                                covered = True
                                break
                        if not covered:
                            cur.is_compound = True
                            cur.compound_partner = nx
                            res.append(cur)
                            i += 2
                            continue
                res.append(cur)
                i += 1
        return res


# --------------------------------------------------------------------------
# writers (TandemRepeat.to_* bwt.py:454-641, save_results bwt.py:4141-4198)
# --------------------------------------------------------------------------
def _fmt_strfinder(r: Rec, marker: str, fl: str, fr: str) -> str:
    if r.is_compound and r.compound_partner is not None:
        p = r.compound_partner
        c1, c2 = r.cons, p.cons
        k1, k2 = int(round(r.copies)), int(round(p.copies))
        core = (r.actual_sequence or c1 * k1) + (p.actual_sequence or c2 * k2)
        full = (fl + core + fr) if (fl or fr) else core
        return (f"{marker}\t{r.chrom}:{r.start + 1}-{p.end}\t[{c1}]n+[{c2}]n\t"
                f"{len(c1)}[{c1}]{k1};{len(c2)}[{c2}]{k2},0\t{k1}/{k2}\t{core}\t100%\t-\t"
                f"{k1}:{k2}\t{k1 + k2}\t{full}\t-")
    c = r.cons
    ml = len(c)
    cc = int(math.floor(r.copies + 1e-6))
    gs = f"{ml}[{c}]{cc},{(r.end - r.start) - ml * cc}"
    if abs(r.copies - round(r.copies)) < 1e-6:
        gt = str(int(round(r.copies)))
    else:
        gt = f"{r.copies:.2f}".rstrip("0").rstrip(".")
    core_full = r.actual_sequence if r.actual_sequence else c * int(r.copies)
    core = f"{core_full[:70]}... (x{cc})" if len(core_full) > 150 else core_full
    cov = f"{r.percent_matches:.0f}%" if r.percent_matches is not None else f"{r.confidence * 100:.0f}%"
    var = ";".join(r.variations) if r.variations else "-"
    fc = (fl + core_full + fr) if (fl or fr) else core_full
    full = f"{fc[:250]}...{fc[-200:]}" if len(fc) > 500 else fc
    return (f"{marker}\t{r.chrom}:{r.start + 1}-{r.end}\t[{c}]n\t{gs}\t{gt}\t{core}\t{cov}\t-\t"
            f"{cc}:{r.n_copies_evaluated}\t{r.n_copies_evaluated}\t{full}\t{var}")


def _comp(r: Rec):
    return r.composition or {"A": 25.0, "C": 25.0, "G": 25.0, "T": 25.0}


def render(p: Pipeline, recs: List[Rec], fmt: str = "strfinder") -> str:
    if fmt == "strfinder":
        recs = p.compounds(recs)
    recs = sorted(recs, key=Rec.key)
    out: List[str] = []
    if fmt == "bed":
        out.append("# Tandem Repeats (BED format with imperfect repeat support)\n")
        out.append("# chrom\tstart\tend\tconsensus_motif\tcopies\ttier\tmismatch_rate\tstrand\n")
        for r in recs:
            out.append(f"{r.chrom}\t{r.start}\t{r.end}\t{r.cons}\t{r.copies:.1f}\t{r.tier}\t"
                       f"{r.mismatch_rate:.3f}\t{r.strand}\n")
    elif fmt == "vcf":
        out.append(VCF_HEADER)
        for i, r in enumerate(recs):
            info = ";".join([f"MOTIF={r.motif}", f"CONS_MOTIF={r.cons}", f"COPIES={r.copies:.1f}",
                             f"TIER={r.tier}", f"CONF={r.confidence:.2f}",
                             f"MM_RATE={r.mismatch_rate:.3f}",
                             f"MAX_MM_PER_COPY={r.max_mismatches_per_copy}",
                             f"N_COPIES_EVAL={r.n_copies_evaluated}", f"STRAND={r.strand}"])
            out.append(f"{r.chrom}\t{r.start + 1}\tTR{i}\t.\t<TR>\t.\tPASS\t{info}\n")
    elif fmt == "trf_table":
        out.append("# Tandem Repeats Finder Compatible Table Format\n")
        out.append("# Indices\tPeriod\tCopyNumber\tConsensusSize\tPercentMatches\tPercentIndels\t")
        out.append("Score\tA\tC\tG\tT\tEntropy\n")
        for r in recs:
            c = _comp(r)
            out.append(f"{r.start}--{r.end}\t{len(r.cons)}\t{r.copies:.1f}\t{len(r.cons)}\t"
                       f"{r.percent_matches:.0f}\t{r.percent_indels:.0f}\t{r.score}\t"
                       f"{c['A']:.0f}\t{c['C']:.0f}\t{c['G']:.0f}\t{c['T']:.0f}\t{r.entropy:.2f}\n")
    elif fmt == "trf_dat":
        for r in recs:
            c = _comp(r)
            sq = r.actual_sequence or (r.cons * int(r.copies))
            out.append(f"{r.start} {r.end} {len(r.cons)} {r.copies:.1f} {len(r.cons)} "
                       f"{r.percent_matches:.0f} {r.percent_indels:.0f} {r.score} "
                       f"{c['A']:.0f} {c['C']:.0f} {c['G']:.0f} {c['T']:.0f} "
                       f"{r.entropy:.2f} {r.cons} {sq}\n")
    elif fmt == "strfinder":
        out.append(STRFINDER_HEADER)
        for r in recs:
            fs = p.full.get(r.chrom, "")
            fl = fs[max(0, r.start - 30):r.start] if fs else ""
            fr = fs[r.end:r.end + 30] if fs else ""
            out.append(_fmt_strfinder(r, f"STR_{r.chrom}", fl, fr) + "\n")
    else:
        raise ValueError(fmt)
    return "".join(out)


STRFINDER_HEADER = ("STR_marker\tSTR_position\tSTR_motif\tSTR_genotype_structure\tSTR_genotype\t"
                    "STR_core_seq\tAllele_coverage\tAlleles_ratio\tReads_Distribution(consensused)\t"
                    "STR_depth\tFull_seq\tVariations\n")
VCF_HEADER = (
    "##fileformat=VCFv4.2\n"
    "##INFO=<ID=MOTIF,Number=1,Type=String,Description=\"Original seed motif\">\n"
    "##INFO=<ID=CONS_MOTIF,Number=1,Type=String,Description=\"Consensus motif from all copies\">\n"
    "##INFO=<ID=COPIES,Number=1,Type=Float,Description=\"Number of copies\">\n"
    "##INFO=<ID=TIER,Number=1,Type=Integer,Description=\"Detection tier (1=short, 2=medium/long, 3=very long)\">\n"
    "##INFO=<ID=CONF,Number=1,Type=Float,Description=\"Confidence score\">\n"
    "##INFO=<ID=MM_RATE,Number=1,Type=Float,Description=\"Overall mismatch rate across all copies\">\n"
    "##INFO=<ID=MAX_MM_PER_COPY,Number=1,Type=Integer,Description=\"Maximum mismatches in any single copy\">\n"
    "##INFO=<ID=N_COPIES_EVAL,Number=1,Type=Integer,Description=\"Number of copies evaluated for consensus\">\n"
    "##INFO=<ID=STRAND,Number=1,Type=String,Description=\"Strand of canonical motif (+/-)\">\n"
    "#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\n")


# --------------------------------------------------------------------------
# FASTA loading (TandemRepeatFinder.load_reference bwt.py:3713-3756)
# --------------------------------------------------------------------------
def load_fasta(path: str, flank_trim: int = 30):
    flank_trim = max(0, flank_trim)
    seqs: Dict[str, str] = {}
    full: Dict[str, str] = {}
    offs: Dict[str, int] = {}
    name = None
    buf: List[str] = []

    def flush():
        s = "".join(buf)
        full[name] = s
        if len(s) <= 2 * flank_trim:
            seqs[name], offs[name] = s, 0
        else:
            seqs[name], offs[name] = s[flank_trim:len(s) - flank_trim], flank_trim

    with open(path, "r") as f:
        for line in f:
            line = line.strip()
            if line.startswith(">"):
                if name:
                    flush()
                name = line[1:].split()[0]
                buf = []
            elif line:
                buf.append(line.upper())
    if name:
        flush()
    return seqs, full, offs


def read_long_reads(path: str) -> List[str]:
    """The CLI's FASTA/FASTQ long-read reader (bwt.py:4312-4328): '>'/'@' lines
    start a read, '+' lines are skipped, every other line (FASTQ quality
    lines included) is upper-cased and appended."""
    reads: List[str] = []
    seq = ""
    with open(path, "r") as f:
        for line in f:
            line = line.strip()
            if line.startswith(">") or line.startswith("@"):
                if seq:
                    reads.append(seq)
                    seq = ""
            elif not line.startswith("+"):
                seq += line.upper()
        if seq:
            reads.append(seq)
    return reads


def run_file(path: str, fmt: str = "strfinder", min_copies: int = 3, max_unit_len: int = 120,
             flank_trim: int = 30, tier2: bool = True, show_progress: bool = False,
             strict_scan=None, long_reads: Optional[List[str]] = None) -> str:
    """Whole CLI path (bwt.py:4293-4361) with `strict_scan(seq_bytes, U, min_copies)`
    supplying raw hits (defaults to the C oracle).  long_reads: Tier 3 in
    parallel mode (bwt.py:3917-3924), after all worker records."""
    if strict_scan is None:
        from oracle import strict_scan as _ss

        def strict_scan(b, U, mc):
            return _ss(b, 1, U, 0, mc)
    seqs, full, offs = load_fasta(path, flank_trim)
    p = Pipeline(seqs, full, offs, min_copies)
    raw: List[Rec] = []
    for chrom, s in seqs.items():
        if not tier2:
            continue
        if len(s) > 50_000_000 and not show_progress:
            continue
        U = max(max_unit_len, min(len(s) // min_copies, 1000))
        hits = strict_scan(s.encode("utf-8"), U, min_copies)
        raw.extend(worker_records(chrom, s, hits))
    if long_reads:
        from . import library
        rb = [x.encode("latin-1", errors="replace") for x in long_reads]
        for chrom, s in seqs.items():
            raw.extend(Rec(**d) for d in library.tier3((s + "$").encode("utf-8"), rb, chrom))
    return render(p, p.run(raw), fmt)
