"""Deterministic synthetic FASTA generator.

The reference ships no large-input generator (only the 142 bp
`test_tandem_repeats.py:81-138` toy), so the benchmark contigs are produced
here.  Everything is driven by splitmix64 in counter mode, computed with
explicit uint64 arithmetic, so the bytes are identical on every machine and
numpy version:

* background: i.i.d. uniform ACGT, base i = top 2 bits of mix(bg + (i+1)·γ);
* planted tandem arrays after every gap ~U[200, 2000]: unit length 60 %
  U{1..6}, 30 % U{7..30}, 10 % U{31..120}; copies U{3..30}; random unit;
* optional "imperfect" variant: each base inside a planted array is
  substituted with probability `sub_rate` (C5 uses 0.02);
* optional assembly gaps (`gaps`, a GAP_PROFILES name), laid over the
  result: runs of `N` after every spacing ~U[a, b], their lengths drawn
  log-uniformly by decade (a decade d uniform, then a length uniform in
  [10^d, 10^(d+1)) -- integer arithmetic only), plus single IUPAC `R`/`Y`
  bases.  Every real assembly carries such runs; they take the index's
  general-alphabet suffix sort and the scan's 4-plane path (bwt.py:212-264,
  1921-1999, and the k-mer table's N->A mapping, bwt.py:138-171);
* output: upper case, 60-column lines, headers ``>contig{k}``.
"""
from __future__ import annotations

import hashlib
import os
from typing import Iterable, List, Optional, Tuple

import numpy as np

GAMMA = 0x9E3779B97F4A7C15
MASK64 = (1 << 64) - 1
SEED_BASE = 0x5EED0000
ACGT = np.frombuffer(b"ACGT", dtype=np.uint8)


def _mix_int(z: int) -> int:
    z &= MASK64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & MASK64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & MASK64
    return z ^ (z >> 31)


def _mix_np(z: np.ndarray) -> np.ndarray:
    z = z.astype(np.uint64, copy=False)
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


class _Stream:
    """Sequential splitmix64 stream (output k = mix(state0 + (k+1)·γ))."""

    def __init__(self, seed: int):
        self.state = seed & MASK64

    def next(self) -> int:
        self.state = (self.state + GAMMA) & MASK64
        return _mix_int(self.state)

    def below(self, m: int) -> int:
        return self.next() % m


def _counter_block(seed: int, start: int, count: int) -> np.ndarray:
    idx = np.arange(start + 1, start + count + 1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(seed & MASK64) + idx * np.uint64(GAMMA)
    return _mix_np(z)


# gap profiles: (spacing lo, spacing hi, first decade, last decade) per run
# class, and the spacing range of single IUPAC bases
GAP_PROFILES = {
    # ~1.4 % N in runs of 10 - 999 bp, one R/Y per ~10 kbp
    "n1": dict(runs=[(2_000, 40_000, 1, 2)], iupac=(1, 20_000)),
    # n1 plus long gaps of 10 kbp - 1 Mbp every ~10 Mbp (~4-5 % N at 100 Mbp)
    "n2": dict(runs=[(2_000, 40_000, 1, 2), (3_000_000, 17_000_000, 4, 5)], iupac=(1, 20_000)),
    # n1 plus runs of 5 - 20 kbp (uniform) every 20-60 kbp: the pure-reference gap golden (G300Np)
    "n3": dict(runs=[(2_000, 40_000, 1, 2), (20_000, 60_000, 5_000, 20_000, "uniform")], iupac=(1, 20_000)),
}


def _gap_layout(length: int, seed: int, profile: str) -> Tuple[List[Tuple[int, int]], List[Tuple[int, int]]]:
    """(start, run length) of every N run and (position, byte) of every IUPAC
    base of one contig under a GAP_PROFILES profile."""
    prof = GAP_PROFILES[profile]
    runs = []
    for k, spec in enumerate(prof["runs"]):
        lo, hi, d0, d1 = spec[:4]
        uniform = len(spec) > 4   # (spacing lo, hi, length lo, hi, "uniform")
        rng = _Stream(_mix_int(seed ^ (0x6A90 + k)))
        cur = 0
        while True:
            cur += lo + rng.below(hi - lo + 1)
            if cur >= length:
                break
            if uniform:
                ln = d0 + rng.below(d1 - d0 + 1)
            else:
                d = d0 + rng.below(d1 - d0 + 1)
                ln = 10 ** d + rng.below(9 * 10 ** d)
            ln = min(ln, length - cur)
            runs.append((cur, ln))
            cur += ln
    iup = []
    lo, hi = prof["iupac"]
    rng = _Stream(_mix_int(seed ^ 0x1A9C))
    cur = 0
    while True:
        cur += lo + rng.below(hi - lo + 1)
        if cur >= length:
            break
        iup.append((cur, b"RY"[rng.below(2)]))
    return runs, iup


def generate_contig(length: int, index: int, sub_rate: float = 0.0,
                    plants: Optional[List[Tuple[int, int, int]]] = None, gaps: Optional[str] = None) -> bytes:
    """Return the sequence bytes of synthetic contig `index`.

    `plants`, when given, receives (start, unit_len, copies) per planted array.
    `gaps` names a GAP_PROFILES entry laid over the contig (None: ACGT only).
    """
    seed = SEED_BASE + index
    bg_seed = _mix_int(seed ^ 0xB6)
    pl_seed = _mix_int(seed ^ 0x91A7)
    sub_seed = _mix_int(seed ^ 0x5B5)

    seq = np.empty(length, dtype=np.uint8)
    chunk = 1 << 22
    for s in range(0, length, chunk):
        c = min(chunk, length - s)
        seq[s:s + c] = ACGT[(_counter_block(bg_seed, s, c) >> np.uint64(62)).astype(np.intp)]

    rng = _Stream(pl_seed)
    cur = 0
    sub_thresh = int(sub_rate * float(1 << 64)) if sub_rate > 0 else 0
    while True:
        cur += 200 + rng.below(1801)
        if cur >= length:
            break
        u = rng.below(100)
        if u < 60:
            unit = 1 + rng.below(6)
        elif u < 90:
            unit = 7 + rng.below(24)
        else:
            unit = 31 + rng.below(90)
        copies = 3 + rng.below(28)
        motif = bytearray()
        while len(motif) < unit:
            w = rng.next()
            for k in range(32):
                if len(motif) == unit:
                    break
                motif.append(b"ACGT"[(w >> (62 - 2 * k)) & 3])
        span = min(unit * copies, length - cur)
        arr = np.frombuffer(bytes(motif) * copies, dtype=np.uint8)[:span]
        seq[cur:cur + span] = arr
        if sub_thresh:
            r = _counter_block(sub_seed, cur, span)
            hit = r < np.uint64(sub_thresh)
            if hit.any():
                code = np.searchsorted(ACGT, seq[cur:cur + span][hit])
                shift = 1 + ((r[hit] >> np.uint64(8)) % np.uint64(3)).astype(np.intp)
                seg = seq[cur:cur + span]
                seg[hit] = ACGT[(code + shift) % 4]
        if plants is not None:
            plants.append((cur, unit, copies))
        cur += span
    if gaps:
        runs, iup = _gap_layout(length, seed, gaps)
        for p, b in iup:
            seq[p] = b
        for s0, ln in runs:
            seq[s0:s0 + ln] = ord("N")
    return seq.tobytes()


def shared_prefix_runs(alphabet: bytes = b"ACGT", seed: int = 1,
                       run_lengths: Iterable[int] = tuple(range(16, 34)) + (40, 48, 63, 64, 65, 100),
                       prefix_lengths: Iterable[int] = (16, 32, 48, 64)) -> bytes:
    """A suffix-sort stress text: for every run symbol c, run length r and
    prefix length p, one random p-base prefix Z (not ending in c) is repeated
    with c^r and then every other symbol x, each copy followed by its own
    random tail -- Z c^r x W.  Two such suffixes share p + r symbols, differ at
    x, and their tails W order them the other way about half of the time, so a
    sort that treats the run's rank as resolving more symbols than it does
    (h-prefix claims of the doubling rounds) orders them by W.  Real genomes
    hold the same pattern: near-identical repeat copies followed by poly-A
    tails of equal length."""
    rng = _Stream(_mix_int(SEED_BASE ^ 0x5A11 ^ seed))

    def rnd(k: int, avoid_last: int = -1) -> bytes:
        b = bytearray(alphabet[rng.below(len(alphabet))] for _ in range(k))
        while k and b[-1] == avoid_last:
            b[-1] = alphabet[rng.below(len(alphabet))]
        return bytes(b)
    parts = [rnd(64)]
    for c in alphabet:
        for r in run_lengths:
            for p in prefix_lengths:
                z = rnd(p, c)
                for x in alphabet:
                    if x != c:
                        parts.append(z + bytes([c]) * r + bytes([x]) + rnd(24))
    return b"".join(parts)


def format_fasta_record(name: str, seq: bytes, width: int = 60) -> bytes:
    arr = np.frombuffer(seq, dtype=np.uint8)
    full = len(arr) // width
    out = [b">" + name.encode() + b"\n"]
    if full:
        body = np.empty((full, width + 1), dtype=np.uint8)
        body[:, :width] = arr[:full * width].reshape(full, width)
        body[:, width] = 10
        out.append(body.tobytes())
    if len(arr) % width:
        out.append(arr[full * width:].tobytes() + b"\n")
    return b"".join(out)


def write_fasta(path: str, lengths: Iterable[int], sub_rate: float = 0.0,
                first_index: int = 1, gaps: Optional[str] = None) -> str:
    """Write contigs ``contig{k}`` (k from `first_index`); return sha256 of the file."""
    h = hashlib.sha256()
    tmp = path + ".tmp"
    with open(tmp, "wb") as f:
        for k, n in enumerate(lengths, first_index):
            rec = format_fasta_record(f"contig{k}", generate_contig(n, k, sub_rate, gaps=gaps))
            h.update(rec)
            f.write(rec)
    os.replace(tmp, path)
    return h.hexdigest()


CONFIGS = {
    # BASELINE.json configs
    "C2": dict(lengths=[1_000_000], sub_rate=0.0),
    "C3": dict(lengths=[100_000_000], sub_rate=0.0),
    "C4": dict(lengths=[12_500_000] * 8, sub_rate=0.0),
    "C5": dict(lengths=[100_000_000], sub_rate=0.02),
    # general alphabet: C3 / one C4 contig with assembly gaps (N runs, R/Y)
    "C3N": dict(lengths=[100_000_000], sub_rate=0.0, gaps="n2"),
    "G12N": dict(lengths=[12_500_000], sub_rate=0.0, gaps="n2", first_index=2),
}


def main(argv=None) -> int:
    import argparse
    ap = argparse.ArgumentParser(description="seeded synthetic FASTA (splitmix64)")
    ap.add_argument("out")
    ap.add_argument("--config", choices=sorted(CONFIGS))
    ap.add_argument("--lengths", type=lambda s: [int(x) for x in s.split(",")])
    ap.add_argument("--sub-rate", type=float, default=None)
    ap.add_argument("--first-index", type=int, default=1)
    ap.add_argument("--gaps", choices=sorted(GAP_PROFILES))
    a = ap.parse_args(argv)
    if a.config:
        cfg = dict(CONFIGS[a.config])
    else:
        cfg = dict(lengths=a.lengths or [1_000_000], sub_rate=0.0)
    if a.sub_rate is not None:
        cfg["sub_rate"] = a.sub_rate
    if a.gaps:
        cfg["gaps"] = a.gaps
    print(write_fasta(a.out, cfg["lengths"], cfg["sub_rate"], a.first_index, cfg.get("gaps")))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
