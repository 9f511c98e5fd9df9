"""Pure-Python restatement of the reference's LIBRARY finders that are not on
the CLI path -- TEST INFRASTRUCTURE (see oracle/__init__), small inputs only.

Reference: /root/reference/bwt.py (wyim-pgl/bwt-algorithm @ 2025-11-14).

  short_imperfect   Tier2LCPFinder.find_short_imperfect_repeats (bwt.py:2027-2095)
                    -> _find_tandems_fm_with_mismatches (2562-2695)
                    -> _extend_tandem_fm (2697-2805), _is_maximal_fm (2807-2825)
                    (FM/k-mer seeds + Hamming
                    seed-and-extend + majority-vote consensus)
  lcp_plateaus      Tier2LCPFinder._detect_lcp_plateaus (2118-2145)
                    -> _analyze_sa_interval_for_tandems (2500-2549),
                    _validate_periodicity_arr (2551-2560)   (A2-9)
  tier1_find_strs   Tier1STRFinder.find_strs (1426-1538)    (§8(f) #2)
  find_repeats_simple  Tier2LCPFinder.find_long_repeats -> _find_repeats_simple
                    (2097-2106, 2177-2390) with _extend_with_mismatches
                    (2392-2498): adaptive period/position scan with
                    majority-vote extension (§8(f) #4; the reference's 30 s
                    wall-clock stop is not restated)
  tier3             Tier3LongReadFinder.find_very_long_repeats (2837-3036):
                    500-byte windows every 100 bytes of each read >= 1000,
                    self-periodicity 10..165, unique 50-byte anchor -> FM
                    locate, consensus/statistics/variations, consolidation
                    (§8(f) #3)

Records are dicts with the reference TandemRepeat field names (bwt.py:429-452).
"""
from __future__ import annotations

import math
from collections import Counter
from itertools import product
from typing import Dict, List, Optional

import numpy as np

from . import post

_TRANSITIONS = {("A", "G"), ("G", "A"), ("C", "T"), ("T", "C")}


def _rec(chrom, start, end, motif, copies, length, tier, confidence=1.0, consensus_motif=None,
         mismatch_rate=0.0, max_mm=0, n_eval=0, strand="+", pm=0.0, pi=0.0, score=0,
         composition=None, entropy=0.0, actual=None, variations=None) -> Dict:
    return dict(chrom=chrom, start=start, end=end, motif=motif, copies=copies, length=length, tier=tier,
                confidence=confidence, consensus_motif=consensus_motif, mismatch_rate=mismatch_rate,
                max_mismatches_per_copy=max_mm, n_copies_evaluated=n_eval, strand=strand,
                percent_matches=pm, percent_indels=pi, score=score, composition=composition,
                entropy=entropy, actual_sequence=actual, variations=variations)


def entropy(s: str) -> float:                       # bwt.py:730-745 (np.log2, Counter order)
    if not s:
        return 0.0
    n = len(s)
    e = 0.0
    for c in Counter(s).values():
        p = c / n
        e -= p * float(np.log2(p))
    return e


def trf_statistics(t: bytes, start: int, end: int, cons: str, copies: int, mm: float):   # 1336-1366
    actual = t[start:end].decode("ascii", errors="replace") if end <= len(t) else cons * int(copies)
    return ((1.0 - mm) * 100.0, 0.0, post.trf_score(end - start, mm), post.composition(cons),
            post.entropy(cons), actual)


def max_mismatches_for_array(motif_len: int, n_copies: int) -> int:   # bwt.py:2003-2025
    total = motif_len * n_copies
    if motif_len == 1:
        return 0
    if motif_len <= 6:
        return max(1, int(np.ceil(0.05 * total)))
    return max(1, int(np.ceil(0.08 * total)))


def _is_transition(b1: int, b2: int) -> bool:      # count_transversions_array, bwt.py:781-800
    c1 = chr(b1) if 65 <= b1 <= 84 else "N"
    c2 = chr(b2) if 65 <= b2 <= 84 else "N"
    return c1 == c2 or (c1, c2) in _TRANSITIONS


def _majority(copies: List[bytes], L: int) -> bytes:
    """np.unique + argmax per column: the smallest byte among the most frequent."""
    out = bytearray(L)
    for p in range(L):
        cnt = Counter(c[p] for c in copies if p < len(c))
        best = max(cnt.values())
        out[p] = min(b for b, v in cnt.items() if v == best)
    return bytes(out)


def extend(t: bytes, seed: int, L: int):           # _extend_tandem_fm, bwt.py:2697-2805
    n = len(t)
    start, end, copies = seed, seed + L, 1

    def mm_transv(s, e, cons):
        tot = tv = 0
        for i in range((e - s) // L):
            a = s + i * L
            if a + L <= n:
                cp = t[a:a + L]
                for x, y in zip(cp, cons):
                    if x != y:
                        tot += 1
                        if not _is_transition(x, y):
                            tv += 1
        return tot, tv

    while end + L <= n:
        nxt = t[end:end + L]
        if L > 1 and len(set(nxt)) == 1:
            break
        tc = copies + 1
        cps = [t[start + i * L:start + i * L + L] for i in range(tc) if start + i * L + L <= n]
        cons = _majority(cps, L)
        tot, tv = mm_transv(start, end + L, cons)
        if tot <= max_mismatches_for_array(L, tc) and tv == 0:
            copies, end = tc, end + L
        else:
            break
    while start - L >= 0:
        prv = t[start - L:start]
        if L > 1 and len(set(prv)) == 1:
            break
        tc = copies + 1
        ts = start - L
        cps = [t[ts + i * L:ts + i * L + L] for i in range(tc) if ts + i * L + L <= n]
        cons = _majority(cps, L)
        tot, tv = mm_transv(ts, end, cons)
        if tot <= max_mismatches_for_array(L, tc) and tv == 0:
            copies, start = tc, ts
        else:
            break
    return start, end, copies


def consensus_array(t: bytes, start: int, L: int, n_copies: int):   # bwt.py:1208-1256
    if n_copies == 0 or L == 0:
        return b"", 0.0, 0
    cps = []
    for i in range(n_copies):
        a = start + i * L
        if a + L > len(t):
            break
        cps.append(t[a:a + L])
    if not cps:
        return b"", 0.0, 0
    cons = _majority(cps, L)
    tot = mx = 0
    for c in cps:
        h = sum(1 for x, y in zip(c, cons) if x != y)
        tot += h
        mx = max(mx, h)
    return cons, tot / (len(cps) * L), mx


def kmer_positions(idx, kmer: str) -> List[int]:   # BWTCore.get_kmer_positions, bwt.py:173-193
    if len(kmer) > 8 or idx.kmer_offsets[-1] == 0:
        return locate(idx, kmer)
    w = 0
    for ch in kmer.upper():
        b = {"A": 0, "C": 1, "G": 2, "T": 3, "N": 0}.get(ch)
        if b is None:
            return []
        w = (w << 2) | b
    return idx.kmer_positions(w)


def locate(idx, pattern: str) -> List[int]:        # bwt.py:398-410
    sp, ep = idx.backward_search(pattern.encode())
    if sp == -1:
        return []
    return sorted(idx.sa[sp:ep + 1].tolist())


_OCC: Dict = {}


def _locate_exact(t: bytes, pattern: str) -> List[int]:
    """locate_positions(pattern) (bwt.py:398-410) = every occurrence of the
    pattern in the index text, ascending; answered from a table of all windows
    of that length (built once per text and length)."""
    k = len(pattern)
    key = (id(t), k)
    tab = _OCC.get(key)
    if tab is None:
        tab = {}
        for i in range(len(t) - k + 1):
            tab.setdefault(t[i:i + k], []).append(i)
        _OCC.clear()
        _OCC[key] = tab
    return tab.get(pattern.encode(), [])


_MOTIFS: Dict = {}


def enumerate_motifs(k: int, alphabet: str = "ACGT"):   # bwt.py:1369-1381
    """Product order; kept iff s == min(rotations) and s is primitive.  For the
    sorted ACGT alphabet, strings compare like their base-4 codes, so a numpy
    pass over all 4^k codes decides both (a rotation < s: not canonical; a
    non-trivial rotation == s: not primitive)."""
    key = (k, alphabet)
    if key not in _MOTIFS:
        if alphabet == "ACGT" and 1 <= k <= 10:
            codes = np.arange(4 ** k, dtype=np.int64)
            keep = np.ones(codes.size, dtype=bool)
            for r in range(1, k):
                hi = codes >> (2 * (k - r))                      # first r symbols
                rot = ((codes & ((1 << (2 * (k - r))) - 1)) << (2 * r)) | hi
                keep &= rot > codes
            res = []
            for cde in codes[keep].tolist():
                res.append("".join("ACGT"[(cde >> (2 * (k - 1 - j))) & 3] for j in range(k)))
        else:
            res = ["".join(tup) for tup in product(alphabet, repeat=k)
                   if post.min_rotation("".join(tup)) == "".join(tup)
                   and post.smallest_period("".join(tup)) == k]
        _MOTIFS[key] = res
    return iter(_MOTIFS[key])


def short_imperfect(chrom: str, t: bytes, idx, min_period: int = 1, max_short_motif: int = 9,
                    min_copies: int = 3, min_array_length: int = 6, min_entropy: float = 1.0,
                    allow_mismatches: bool = True, tier1_seen=()) -> List[Dict]:
    """find_short_imperfect_repeats(chromosome, tier1_seen) on text t (incl. '$')."""
    out: List[Dict] = []
    n = len(t)
    if n > 1_000_000:
        return out
    _EXT_CACHE.clear()       # both caches are keyed by id(t): never reuse them across calls
    _OCC.clear()
    seen = np.zeros(n + 1, dtype=bool)
    for s, e in tier1_seen:                        # `any(start <= p < end ...)` as a bitmap
        seen[max(0, s):max(0, min(n, e))] = True
    for k in range(min_period, min(max_short_motif + 1, 10)):
        for motif in enumerate_motifs(k):
            if entropy(motif) < min_entropy:
                continue
            rc = post.revcomp(motif)
            rots = set([motif[i:] + motif[:i] for i in range(len(motif))] +
                       [rc[i:] + rc[:i] for i in range(len(rc))])
            allpos = []
            for r in rots:
                allpos.extend(kmer_positions(idx, r) if k <= 8 else _locate_exact(t, r))
            positions = sorted(set(allpos))
            if len(positions) >= min_copies and allow_mismatches:
                _fm_with_mismatches(chrom, t, positions, k, seen, min_copies, min_array_length, out)
    return out


_EXT_CACHE: Dict = {}


def _extend_cached(t: bytes, cs: int, L: int):
    """extend() depends only on (text, start, unit length): memoised per text."""
    key = (id(t), cs, L)
    r = _EXT_CACHE.get(key)
    if r is None:
        r = _EXT_CACHE[key] = extend(t, cs, L)
    return r


def _fm_with_mismatches(chrom, t, positions, motif_len, seen, min_copies, min_array_length, out):
    n = len(t)                                     # _find_tandems_fm_with_mismatches, 2562-2695
    for seed in sorted(positions):
        if seen[seed]:
            continue
        if seed + motif_len > n:
            continue
        best = None
        for shift in range(min(motif_len, seed + 1)):
            cs = seed - shift
            ce = cs + motif_len
            if cs < 0 or ce > n or seen[cs]:
                continue
            s, e, c = _extend_cached(t, cs, motif_len)
            if not (s <= seed < e):
                continue
            if best is None or c > best[2] or (c == best[2] and s < best[0]):
                best = (s, e, c)
        if best is None:
            continue
        start, end, copies = best
        if copies >= min_copies and end - start >= min_array_length:
            cons, mm, mx = consensus_array(t, start, motif_len, copies)
            if not cons:
                continue
            cs_ = cons.decode("ascii", errors="replace")
            p = post.smallest_period(cs_)
            if p < len(cs_):
                motif_len = p                      # persists for the later seeds (reference quirk)
                copies = max(1, (end - start) // motif_len)
                end = start + copies * motif_len
                cons, mm, mx = consensus_array(t, start, motif_len, copies)
                if not cons:
                    continue
                cs_ = cons.decode("ascii", errors="replace")
            _, strand = post.canonical_stranded(cs_)
            maximal = not ((start > 0 and t[start - 1] == cons[motif_len - 1]) or
                           (end < n and t[end] == cons[0]))
            if maximal:
                conf = max(0.5, 1.0 - mm)
                pm, pi, sc, comp, ent, act = trf_statistics(t, start, end, cs_, copies, mm)
                if pm < (90.0 if motif_len <= 6 else 85.0):
                    continue
                if pi > 5.0:
                    continue
                seq = t.decode("ascii", errors="replace")
                summ = post.align_region(seq, start, end, cs_, 0.1, None, 1) if end > start else None
                var = summ["variations"] if summ else []
                out.append(_rec(chrom, start, end, cs_, copies, end - start, 2, conf, cs_, mm, mx, copies,
                                strand, pm, pi, sc, comp, ent, act, var if var else None))
                seen[start:end] = True


def lcp_plateaus(chrom: str, t: bytes, sa: np.ndarray, lcp: np.ndarray, min_period: int = 1,
                 max_period: int = 1000, min_copies: int = 3) -> List[Dict]:
    out: List[Dict] = []
    n = len(lcp)
    if n == 0:
        return out
    lmax = int(lcp.max())
    if lmax < min_period:
        return out
    thr = max(min_period, min(min(max_period, lmax), 20))
    i = 0
    while i < n:
        if lcp[i] >= thr:
            j = i
            while j < n and lcp[j] >= thr:
                j += 1
            pos = sorted(int(x) for x in sa[i:j])
            for a in range(len(pos)):
                copies, sp = 1, pos[a]
                b = a + 1
                while b < len(pos) and pos[b] == sp + copies * thr:
                    copies += 1
                    b += 1
                if copies >= min_copies and sp + thr <= len(t):
                    motif = t[sp:sp + thr]
                    rep = t[sp:sp + copies * thr]
                    m = len(rep)
                    if m >= 2 * thr:
                        match = sum(1 for q in range(m) if rep[q] == motif[q % thr])
                        if match / m >= 0.8:
                            out.append(_rec(chrom, sp, sp + copies * thr, motif.decode("ascii"), copies,
                                            copies * thr, 2, 0.9))
            i = j
        else:
            i += 1
    return out


def tier1_find_strs(chrom: str, t: bytes, max_motif_length: int = 9, min_copies: int = 3,
                    min_array_length: int = 6, min_entropy: float = 1.0) -> List[Dict]:
    out: List[Dict] = []
    n = len(t)
    seen = np.zeros(n + 1, dtype=bool)
    step = 50 if n > 10_000_000 else (20 if n > 5_000_000 else 1)
    for L in range(min(max_motif_length, 9), 0, -1):
        i = 0
        while i < n - L:
            if seen[i]:
                i += step
                continue
            motif_b = t[i:i + L]
            motif = motif_b.decode("ascii", errors="replace")
            if not all(c in "ACGT" for c in motif):
                i += step
                continue
            copies, cp = 1, i + L
            while cp + L <= n and t[cp:cp + L] == motif_b:
                copies += 1
                cp += L
            if copies >= min_copies:
                end = i + copies * L
                length = end - i
                if entropy(motif) < min_entropy and length < 10:
                    i += step
                    continue
                if length >= min_array_length:
                    pm, pi, sc, comp, ent, act = trf_statistics(t, i, end, motif, copies, 0.0)
                    out.append(_rec(chrom, i, end, motif, float(copies), length, 1, 1.0, motif, 0.0, 0, copies,
                                    "+", pm, pi, sc, comp, ent, t[i:end].decode("ascii", errors="replace")))
                    seen[i:end] = True
                    i = end
                    continue
            i += step
    return out


# ------------------------------------------------------------------ Tier 3
def _t3_structure(window: bytes):
    """_detect_repetitive_structure + _score_periodicity (bwt.py:2948-2984):
    the first period 10 <= p < len // 3 with the highest score > 0.7, where
    score = #{i : w[i] == w[i % p]} / len(w) (motif = w[:p] covers every i)."""
    if len(window) < 50:
        return None
    w = np.frombuffer(window, dtype=np.uint8)
    idx = np.arange(len(w))
    best_p, best_copies, best_score = None, 0, 0
    for p in range(10, len(w) // 3):
        score = int(np.count_nonzero(w == w[idx % p])) / len(w)
        if score > best_score and score > 0.7:
            best_score, best_p, best_copies = score, p, len(w) // p
    if best_p and best_copies >= 3:
        return window[:best_p], best_copies, best_score
    return None


def _t3_map(idx, read: bytes, position: int) -> int:   # _map_read_to_reference, bwt.py:2986-3001
    anchor_start = max(0, position - 50)
    anchor = read[anchor_start:position]
    if len(anchor) >= 20:
        sp, ep = idx.backward_search(anchor)
        if sp != -1 and ep == sp:
            return int(idx.sa[sp]) + (position - anchor_start)
    return -1


def tier3(text: bytes, reads: List[bytes], chromosome: str, idx=None) -> List[Dict]:
    """Tier3LongReadFinder(BWTCore(text)).find_very_long_repeats(reads, chromosome)
    (bwt.py:2837-2850 -> _analyze_read_for_repeats 2852-2946 ->
    _consolidate_repeat_calls 3003-3036).  text includes the sentinel."""
    from . import Index
    idx = idx if idx is not None else Index(text)
    max_len = len(text) - 1 if text and text[-1] == 36 else len(text)   # 2877-2880
    seq = text.decode("ascii", errors="replace")
    reps: List[Dict] = []
    for read in reads:
        if len(read) < 1000:                                               # 2842
            continue
        for start in range(0, len(read) - 500, 100):                       # 2857-2861
            info = _t3_structure(read[start:start + 500])
            if not info:
                continue
            motif, copies, confidence = info
            ref_start = _t3_map(idx, read, start)
            if ref_start < 0:
                continue
            motif_len = len(motif)
            if ref_start >= max_len:
                continue
            avail = max((max_len - ref_start) // motif_len, 0)
            if avail == 0:
                continue
            copies_int = max(1, min(int(round(copies)), avail))
            ref_end = ref_start + motif_len * copies_int
            cons = motif.decode("ascii", errors="replace")
            mm, max_mm = 0.0, 0
            pm, pi, score = 100.0, 0.0, 0
            comp, ent = post.composition(cons), entropy(cons)
            actual = (cons * copies_int)[:max(ref_end - ref_start, 0)]
            if motif_len > 0 and ref_end > ref_start:
                carr, mm, max_mm = consensus_array(text, ref_start, motif_len, copies_int)
                if carr:
                    cons = carr.decode("ascii", errors="replace")
                    motif_len = len(cons)
                if ref_end <= max_len:
                    pm, pi, score, comp, ent, actual = trf_statistics(text, ref_start, ref_end, cons, copies_int, mm)
            _, strand = post.canonical_stranded(cons)
            var = None                                                     # summarize_variations_array (1259-1287)
            if len(text) and motif_len > 0:
                s0, e0 = max(0, ref_start), min(len(seq), ref_end if ref_end > ref_start else len(seq))
                if e0 > s0:
                    summ = post.align_region(seq, s0, e0, cons, 0.1, None, 1)
                    if summ and summ["variations"]:
                        var = summ["variations"]
            reps.append(_rec(chromosome, ref_start, ref_end, cons, float(copies_int), ref_end - ref_start, 3,
                             confidence, cons, mm, max_mm, copies_int, strand, pm, pi, score, comp, ent,
                             actual, var))
    if not reps:
        return reps
    reps.sort(key=lambda r: (post.natural_key(r["chrom"]), r["start"], r["end"]))
    out, cur = [], reps[0]
    for r in reps[1:]:
        if r["chrom"] == cur["chrom"] and r["start"] <= cur["end"] and r["motif"] == cur["motif"]:
            s, e = min(cur["start"], r["start"]), max(cur["end"], r["end"])
            cur = _rec(cur["chrom"], s, e, cur["motif"], (cur["copies"] + r["copies"]) / 2, e - s, cur["tier"],
                       min(cur["confidence"], r["confidence"]))
        else:
            out.append(cur)
            cur = r
    out.append(cur)
    return out


# ------------------------------------------------- simple period scan
def _smallest_period_kmp(a: bytes) -> int:          # _smallest_period_codes, bwt.py:2161-2175
    n = len(a)
    if n == 0:
        return 0
    pi = [0] * n
    j = 0
    for i in range(1, n):
        while j > 0 and a[i] != a[j]:
            j = pi[j - 1]
        if a[i] == a[j]:
            j += 1
        pi[i] = j
    p = n - pi[-1]
    return p if p != 0 and n % p == 0 else n


def _majority_full(cps: List[bytes], L: int) -> bytes:
    out = bytearray(L)
    for pos in range(L):
        cnt = Counter(c[pos] for c in cps if pos < len(c))
        if cnt:
            best = max(cnt.values())
            out[pos] = min(b for b, v in cnt.items() if v == best)
    return bytes(out)


def extend_with_mismatches(t: bytes, start_pos: int, period: int, n: int, allow: bool):
    """_extend_with_mismatches (bwt.py:2392-2498) -> (array_start, array_end,
    copies, full_start, full_end)."""
    motif = t[start_pos:start_pos + period]
    start, end, copies = start_pos, start_pos + period, 1
    consensus = motif

    def total_mm(s, e, cons):
        tot = 0
        for i in range((e - s) // period):
            a = s + i * period
            if a + period <= n:
                tot += sum(1 for x, y in zip(t[a:a + period], cons) if x != y)
        return tot

    while end + period <= n:
        tc = copies + 1
        cps = [t[start + i * period:start + i * period + period] for i in range(tc)
               if start + i * period + period <= n]
        cons = _majority_full(cps, period)
        mx = max_mismatches_for_array(period, tc) if allow else 0
        if total_mm(start, end + period, cons) <= mx:
            copies, end, consensus = tc, end + period, cons
        else:
            break
    while start - period >= 0:
        tc = copies + 1
        ts = start - period
        cps = [t[ts + i * period:ts + i * period + period] for i in range(tc) if ts + i * period + period <= n]
        cons = _majority_full(cps, period)
        mx = max_mismatches_for_array(period, tc) if allow else 0
        if total_mm(ts, end, cons) <= mx:
            copies, start, consensus = tc, ts, cons
        else:
            break
    fs, fe = start, end
    pr = 0
    while pr < period and fe + pr < n:
        if t[fe + pr] != consensus[pr % period]:
            break
        pr += 1
    pl = 0
    while pl < period and fs - pl - 1 >= 0:
        if t[fs - pl - 1] != consensus[period - 1 - (pl % period)]:
            break
        pl += 1
    return fs - pl, fe + pr, copies, fs, fe


def find_repeats_simple(chromosome: str, text: bytes, tier1_seen=(), min_period: int = 1,
                        max_period: int = 1000, allow_mismatches: bool = True, min_entropy: float = 1.0,
                        min_copies: int = 3, min_array_length: int = 6, max_iterations: int = 100_000):
    """Tier2LCPFinder._find_repeats_simple (bwt.py:2177-2390) behind
    find_long_repeats (2097-2106).  The reference also stops after 30 s of
    wall time (2238-2257), which makes its output machine-dependent; this
    restatement (like the device path) never times out -- it is the
    reference's result whenever the reference finishes within its limit."""
    n = len(text)
    if n > 0 and text[n - 1] == 36:
        n -= 1
    max_p = min(max_period, max(1, n // 2))
    if n > 100_000:
        max_p = min(max_p, 30)
    elif n > 10_000:
        max_p = min(max_p, 50)
    elif n > 1_000:
        max_p = min(max_p, 100)
    else:
        max_p = min(max_p, 200)
    min_p = min(min_period, max_p)
    mask = bytearray(n)
    for s, e in tier1_seen:
        for x in range(max(0, s), min(e, n)):
            mask[x] = 1
    if n > 10_000_000:
        step, pstep = 500, 20
    elif n > 5_000_000:
        step, pstep = 200, 10
    elif n > 1_000_000:
        step, pstep = 100, 5
    elif n > 100_000:
        step, pstep = 50, 2
    elif n > 10_000:
        step, pstep = 20, 1
    else:
        step, pstep = 10, 1
    results, seen = [], set()
    it = 0
    for p in range(min_p, max_p + 1, pstep):
        i = 0
        while i + 2 * p <= n:
            it += 1
            if it > max_iterations:
                return results
            if i < n and mask[i]:
                i += step
                continue
            mv = text[i:i + p]
            if 36 in mv or 78 in mv:
                i += step
                continue
            if entropy(mv.decode("ascii", errors="replace")) < min_entropy:
                i += step
                continue
            a_s, a_e, cf, fs, fe = extend_with_mismatches(text, i, p, n, allow_mismatches and p <= 64)
            alen = a_e - a_s
            if alen < min_array_length:
                i += step
                continue
            part = max(0, alen - cf * p)
            pf = part / p if p > 0 else 0.0
            eff_i = cf + (1 if pf >= 0.75 else 0)
            if cf >= min_copies or eff_i >= min_copies:
                mv = text[fs:fs + p]
                prim = _smallest_period_kmp(mv)
                pe = prim if prim < p else p
                a_s, a_e, cf, fs, fe = extend_with_mismatches(text, fs, pe, n, allow_mismatches and pe <= 64)
                alen = a_e - a_s
                part = max(0, alen - cf * pe)
                pf = part / pe if pe > 0 else 0.0
                eff_i = cf + (1 if pf >= 0.75 else 0)
                eff_f = cf + pf
                if cf < min_copies and eff_i < min_copies:
                    i += step
                    continue
                carr, mm, mxm = consensus_array(text, fs, pe, cf)
                if not carr:
                    i += step
                    continue
                cons = carr.decode("ascii", errors="replace")
                pl = post.smallest_period(cons)
                if pl < len(cons):
                    pe = pl
                    cf = max(1, (a_e - a_s) // pe)
                    a_e = a_s + cf * pe
                    carr, mm, mxm = consensus_array(text, a_s, pe, cf)
                    if not carr:
                        i += step
                        continue
                    cons = carr.decode("ascii", errors="replace")
                canon, strand = post.canonical_stranded(cons)
                key = (a_s, a_e, canon)
                if key not in seen:
                    seen.add(key)
                    conf = max(0.5, 0.95 - mm)
                    pm, pi, sc, comp, ent, act = trf_statistics(text, a_s, a_e, cons, eff_f, mm)
                    var = None
                    seq = text.decode("ascii", errors="replace")
                    s0, e0 = max(0, a_s), min(len(seq), a_e if a_e > a_s else len(seq))
                    if e0 > s0 and pe > 0:
                        summ = post.align_region(seq, s0, e0, cons, 0.1, None, 1)
                        if summ and summ["variations"]:
                            var = summ["variations"]
                    results.append(_rec(chromosome, a_s, a_e, cons, float(cf), a_e - a_s, 2, conf, cons, mm, mxm,
                                        cf, strand, pm, pi, sc, comp, ent, act, var))
                i = a_e
            else:
                i += step
    return results
