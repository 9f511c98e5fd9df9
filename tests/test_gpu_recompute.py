"""The merge fold's DP recomputes on the device (csrc/recompute.hip, one
wavefront per region) against the host alignment (motif.cpp, itself pinned by
the reference's align_repeat_region fixtures in motif_known.json and the
full-size goldens): _recompute_repeat's two attempts (bwt.py:3530-3534) of
MotifUtils.align_repeat_region (bwt.py:998-1102) on imperfect tandem repeats
with substitutions, insertions and deletions, every motif length 2..256, the
text-end clamps, and the bounds past which a region comes back to the host.
Integer and string results: exact; the mismatch rate is tot_err / (copies * m)
on both sides, compared exactly."""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

_B = np.frombuffer(b"ACGT", dtype=np.uint8)


def _mutated_repeat(r, unit: bytes, copies: int, sub: float, indel: float) -> bytes:
    out = bytearray()
    for _ in range(copies):
        for b in unit:
            x = r.random()
            if x < indel / 2:
                continue                                   # deletion
            if x < indel:
                out.append(int(_B[r.integers(4)]))         # insertion before the base
            out.append(int(_B[r.integers(4)]) if r.random() < sub else b)
    return bytes(out)


def _case_text(seed: int):
    """A text of planted imperfect repeats; regions as the merge fold asks them:
    (start, end, m) with start on a repeat and end near its end."""
    r = np.random.default_rng(seed)
    text = bytearray()
    regions = []
    for _ in range(60):
        text += bytes(_B[r.integers(0, 4, int(r.integers(0, 40)))])
        m = int(r.choice([2, 3, 4, 5, 6, 7, 8, 10, 12, 16, 20, 25, 31, 40, 48, 64, 80, 100, 128, 200, 256]))
        unit = bytes(_B[r.integers(0, 4, m)])
        copies = int(r.integers(1, 9 if m < 64 else 4))
        sub = float(r.choice([0.0, 0.02, 0.05, 0.12]))
        indel = float(r.choice([0.0, 0.01, 0.03]))
        a = len(text)
        text += unit + _mutated_repeat(r, unit, copies, sub, indel)
        b = len(text)
        end = int(b + r.integers(-m, m + 1))
        regions.append((a, max(a + 1, end), m))
        if r.random() < 0.3:   # a second request inside the repeat
            s2 = int(r.integers(a, max(a + 1, b - m)))
            regions.append((s2, b, m))
    text += bytes(_B[r.integers(0, 4, 30)])
    return bytes(text), regions


def _host(seq: bytes, start: int, end: int, m: int, mc: int):
    from bwtmi import MotifUtils as M
    s = seq.decode()
    tmpl = s[start:start + m]
    got = M.align_repeat_region(s, start, end, tmpl, min_copies=mc)
    if got is None:
        got = M.align_repeat_region(s, start, end, tmpl, min_copies=1)
    if got is None:
        return None
    return (got.copies, got.consumed_length, got.max_errors_per_copy, got.total_insertions,
            got.total_deletions, sum(got.error_counts), got.consensus, ";".join(got.variations))


@pytest.mark.parametrize("seed", [1, 2, 3, 4])
def test_device_recompute_matches_host(gpu_ctx, seed):
    from bwtmi import _lib
    seq, regions = _case_text(seed)
    for mc in (3, 1):
        got = _lib.align_regions(gpu_ctx, seq, regions, mc)
        on_dev = 0
        for (s, e, m), g in zip(regions, got):
            want = _host(seq, s, e, m, mc)
            if g is None:
                assert want is None, (seed, s, e, m)
                continue
            on_dev += g[8]
            assert want is not None and tuple(g[:8]) == want, (seed, s, e, m, g, want)
        assert on_dev >= 0.9 * sum(1 for g in got if g is not None), seed


def test_device_recompute_edges(gpu_ctx):
    """Text-end clamps (limit = len, windows shorter than m), a region reaching
    past the text, exact periodic runs of every phase, one-copy regions, and
    motifs past the device bound (257: aligned on the host, on_device False)."""
    from bwtmi import _lib
    r = np.random.default_rng(7)
    unit = bytes(_B[r.integers(0, 4, 7)])
    seq = bytes(_B[r.integers(0, 4, 11)]) + unit * 40 + unit[:3]
    n = len(seq)
    regions = [(11, n, 7), (11, n + 50, 7), (n - 20, n, 7), (n - 9, n, 7), (12, 40, 7), (11, 12, 7),
               (0, 11, 2), (11, 11 + 7 * 3, 7), (n - 7, n, 7)]
    big = bytes(_B[r.integers(0, 4, 257)])
    seq2 = seq + big * 3 + bytes(_B[r.integers(0, 4, 20)])
    regions2 = regions + [(len(seq), len(seq) + 257 * 3, 257), (len(seq), len(seq) + 256 * 3, 256)]
    got = _lib.align_regions(gpu_ctx, seq2, regions2, 3)
    for (s, e, m), g in zip(regions2, got):
        want = _host(seq2, s, e, m, 3)
        assert (g is None) == (want is None), (s, e, m)
        if g is not None:
            assert tuple(g[:8]) == want, (s, e, m, g, want)
            assert g[8] == (m <= 256), (s, e, m)


def test_device_recompute_reference_fixtures(gpu_ctx, golden_dir):
    """The reference's align_repeat_region fixtures (motif_known.json) whose
    template is the region's first m bases and whose motif has >= 2 bases."""
    from bwtmi import _lib
    with open(os.path.join(golden_dir, "motif_known.json")) as f:
        k = json.load(f)
    n = 0
    for seq, s, e, m, mc, want in k["align"]:
        if len(m) < 2 or seq[max(0, s):max(0, s) + len(m)] != m or len(m) > 256:
            continue
        got = _lib.align_regions(gpu_ctx, seq.encode(), [(s, e, len(m))], mc)[0]
        host = _host(seq.encode(), s, e, len(m), mc)
        assert (got is None) == (host is None)
        if got is not None:
            assert tuple(got[:8]) == host
        if want is not None and got is not None and got[0] >= mc:   # first attempt succeeded
            assert (got[6], got[0], got[1]) == (want["consensus"], want["copies"], want["consumed"])
        n += 1
    assert n > 0
