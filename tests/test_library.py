"""Library finders off the CLI path (§8(f) #2):
short imperfect repeats (FM / k-mer seeds + Hamming seed-and-extend +
majority-vote consensus), LCP plateaus, Tier 1 sliding window.

tests/golden/library.json holds the reference's own outputs (make_goldens.py
library).  CPU tests pin the oracle restatement (oracle/library.py) to them;
GPU tests check the device path against both."""
import json
import os

import numpy as np
import pytest

import oracle
from oracle import library as olib

FIELDS = ("start", "end", "motif", "copies", "length", "tier", "confidence", "consensus_motif",
          "mismatch_rate", "max_mismatches_per_copy", "n_copies_evaluated", "strand", "percent_matches",
          "percent_indels", "score", "composition", "entropy", "actual_sequence", "variations")


@pytest.fixture(scope="module")
def lib_golden(golden_dir):
    path = os.path.join(golden_dir, "library.json")
    if not os.path.exists(path):
        pytest.skip("library.json not generated")
    with open(path) as f:
        return json.load(f)


def _cmp(got, want, fields=FIELDS):
    assert len(got) == len(want)
    for g, w in zip(got, want):
        for k in fields:
            gv, wv = g[k], w[k]
            if isinstance(wv, float) or isinstance(gv, float):
                assert float(gv) == float(wv), (k, g, w)
            else:
                assert gv == wv, (k, g, w)


# --------------------------------------------------------------- oracle vs reference
def test_oracle_short_imperfect_matches_reference(lib_golden):
    for name, case in lib_golden.items():
        t = case["seq"].encode() + b"$"
        got = olib.short_imperfect(name, t, oracle.Index(t))
        _cmp(got, case["short_imperfect"])


def test_oracle_lcp_plateaus_matches_reference(lib_golden):
    for name, case in lib_golden.items():
        t = case["seq"].encode() + b"$"
        idx = oracle.Index(t)
        got = olib.lcp_plateaus(name, t, idx.sa, idx.lcp())
        _cmp(got, case["lcp_plateaus"], ("start", "end", "motif", "copies", "length", "tier", "confidence"))


def test_oracle_tier1_matches_reference(lib_golden):
    for name, case in lib_golden.items():
        t = case["seq"].encode() + b"$"
        _cmp(olib.tier1_find_strs(name, t), case["tier1"])


# --------------------------------------------------------------------- device
DEV_FIELDS = ("start", "end", "motif", "copies", "length", "tier", "confidence", "mismatch_rate",
              "max_mismatches_per_copy", "n_copies_evaluated", "strand", "actual_sequence", "variations")


def _as_dicts(reps):
    return [dict(start=r.start, end=r.end, motif=r.motif, copies=r.copies, length=r.length, tier=r.tier,
                 confidence=r.confidence, mismatch_rate=r.mismatch_rate,
                 max_mismatches_per_copy=r.max_mismatches_per_copy, n_copies_evaluated=r.n_copies_evaluated,
                 strand=r.strand, actual_sequence=r.actual_sequence, variations=r.variations) for r in reps]


def _finder(seq: str):
    from bwtmi import BWTCore
    from bwtmi.tiers import Tier2LCPFinder
    return Tier2LCPFinder(BWTCore(seq + "$"))


@pytest.mark.gpu
def test_device_short_imperfect_matches_reference(gpu_ctx, lib_golden):
    for name, case in lib_golden.items():
        f = _finder(case["seq"])
        _cmp(_as_dicts(f.find_short_imperfect_repeats(name, set())), case["short_imperfect"], DEV_FIELDS)


@pytest.mark.gpu
def test_device_lcp_plateaus_matches_reference(gpu_ctx, lib_golden):
    for name, case in lib_golden.items():
        f = _finder(case["seq"])
        got = f._detect_lcp_plateaus(f._compute_lcp_array(), name)
        _cmp(_as_dicts(got), case["lcp_plateaus"], ("start", "end", "motif", "copies", "length", "tier",
                                                      "confidence"))


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [11, 12, 13, 14])
def test_device_short_imperfect_vs_oracle(gpu_ctx, seed):
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    from make_goldens import _crafted_short
    seq = _crafted_short(seed, 40)
    t = seq + b"$"
    idx = oracle.Index(t)
    want = olib.short_imperfect("c", t, idx)
    assert want
    f = _finder(seq.decode())
    _cmp(_as_dicts(f.find_short_imperfect_repeats("c", set())), want, DEV_FIELDS)
    # tier1_seen regions (bwt.py:2041) are skipped as seeds and candidate starts
    seen = {(w["start"] + 1, w["end"] - 2) for w in want[::2]}
    want2 = olib.short_imperfect("c", t, idx, tier1_seen=seen)
    _cmp(_as_dicts(f.find_short_imperfect_repeats("c", seen)), want2, DEV_FIELDS)


@pytest.mark.gpu
@pytest.mark.parametrize("kw", [dict(min_copies=2, min_array_length=4), dict(min_copies=4, min_array_length=20),
                                dict(min_copies=3, min_array_length=30, min_period=2, max_short_motif=7),
                                dict(min_copies=2, min_array_length=1, min_entropy=0.5),
                                dict(allow_mismatches=False)])
def test_device_short_imperfect_parameters_vs_oracle(gpu_ctx, kw):
    """The finder's thresholds reach the device seed flags (k_seed_flags keeps a
    seed when some window through it has >= max(min_copies, ceil(min_array_length
    / L)) copies): other min_copies / min_array_length / period / entropy
    settings against the oracle."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    from make_goldens import _crafted_short
    seq = _crafted_short(17, 40)
    t = seq + b"$"
    idx = oracle.Index(t)
    want = olib.short_imperfect("c", t, idx, **kw)
    f = _finder(seq.decode())
    for k, v in kw.items():
        setattr(f, k, v)
    _cmp(_as_dicts(f.find_short_imperfect_repeats("c", set())), want, DEV_FIELDS)


@pytest.mark.gpu
def test_device_tier1_matches_reference(gpu_ctx, lib_golden):
    from bwtmi.tiers import Tier1STRFinder
    for name, case in lib_golden.items():
        t = np.frombuffer(case["seq"].encode() + b"$", dtype=np.uint8)
        got = _as_dicts(Tier1STRFinder(t, 9).find_strs(name))
        _cmp(got, case["tier1"], DEV_FIELDS)


@pytest.mark.gpu
@pytest.mark.parametrize("n,mml", [(300_000, 9), (6_000_000, 9), (11_000_000, 6)])
def test_device_tier1_vs_oracle(gpu_ctx, n, mml):
    """Position step 1 / 20 / 50 regimes (n > 5 and > 10 Mbp, bwt.py:1440-1447)."""
    from bwtmi import synth
    from bwtmi.tiers import Tier1STRFinder
    seq = synth.generate_contig(n, 900 + mml, 0.01)
    want = olib.tier1_find_strs("c", seq, mml)
    got = _as_dicts(Tier1STRFinder(np.frombuffer(seq, dtype=np.uint8), mml).find_strs("c"))
    assert len(want) > 0
    _cmp(got, want, DEV_FIELDS)


@pytest.mark.gpu
def test_device_lcp_plateaus_vs_oracle_100kbp(gpu_ctx):
    from bwtmi import synth
    seq = synth.generate_contig(100_000, 77, 0.01)
    t = seq + b"$"
    idx = oracle.Index(t)
    want = olib.lcp_plateaus("c", t, idx.sa, idx.lcp())
    f = _finder(seq.decode())
    got = f._detect_lcp_plateaus(None, "c")
    assert len(want) > 0
    _cmp(_as_dicts(got), want, ("start", "end", "motif", "copies", "length", "tier", "confidence"))
