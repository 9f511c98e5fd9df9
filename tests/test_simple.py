"""Tier2LCPFinder.find_long_repeats -> _find_repeats_simple (SURVEY.md §8(f)
#4; bwt.py:2097-2106, 2177-2498).

tests/golden/simple.json holds the reference's own outputs (make_goldens.py
simple) on seeded, crafted and edge contigs (one with a Tier 1 mask, one
without mismatches, one with a period floor); each case finished well inside
the reference's 30 s wall-clock stop, so that stop never fired and the
outputs are deterministic.  CPU tests pin the oracle restatement
(oracle/library.py find_repeats_simple) to them; GPU tests check the device
path against the goldens and against the oracle, including a 2 Mbp input
that reaches the reference's 100,000-iteration cap."""
import dataclasses
import json
import os

import numpy as np
import pytest

from oracle import library as olib

FIELDS = ("start", "end", "motif", "copies", "length", "tier", "confidence", "consensus_motif",
          "mismatch_rate", "max_mismatches_per_copy", "n_copies_evaluated", "strand", "percent_matches",
          "percent_indels", "score", "composition", "entropy", "actual_sequence", "variations")

_PARAMS = dict(min_period=1, max_period=1000, allow_mismatches=True)


@pytest.fixture(scope="module")
def simple_golden(golden_dir):
    path = os.path.join(golden_dir, "simple.json")
    if not os.path.exists(path):
        pytest.skip("simple.json not generated")
    with open(path) as f:
        return json.load(f)


def _cmp(got, want, fields=FIELDS):
    assert len(got) == len(want), (len(got), len(want))
    for g, w in zip(got, want):
        for k in fields:
            gv, wv = g[k], w[k]
            if isinstance(wv, float) or isinstance(gv, float):
                assert float(gv) == float(wv), (k, g, w)
            else:
                assert gv == wv, (k, g, w)


def _oracle(name, seq: bytes, params, seen):
    kw = dict(_PARAMS, **params)
    return olib.find_repeats_simple(name, seq + b"$", [tuple(x) for x in seen], kw["min_period"],
                                    kw["max_period"], kw["allow_mismatches"])


def _device(name, seq: str, params, seen):
    from bwtmi import BWTCore
    from bwtmi.tiers import Tier2LCPFinder
    kw = dict(_PARAMS, **params)
    f = Tier2LCPFinder(BWTCore(seq + "$"), min_period=kw["min_period"], max_period=kw["max_period"],
                       allow_mismatches=kw["allow_mismatches"])
    out = [dataclasses.asdict(r) for r in f.find_long_repeats(name, {tuple(x) for x in seen})]
    for r in out:
        r.pop("chrom")
    return out


def test_oracle_simple_scan_matches_reference(simple_golden):
    for name, case in simple_golden.items():
        got = _oracle(name, case["seq"].encode(), case["params"], case["tier1_seen"])
        _cmp(got, case["records"])


def test_oracle_extension_known_answers():
    t = b"ACGTACGTACGAACGTACGTTT"
    # right extension absorbs the copy with one substitution (allowance ceil(0.05 * 4c) = 1 up to
    # five copies); the bases after it ('TT') do not start the consensus 'ACGT'
    assert olib.extend_with_mismatches(t, 0, 4, len(t), True) == (0, 20, 5, 0, 20)
    # exact copies only: two full copies, then 'ACG' of the third as a partial copy
    assert olib.extend_with_mismatches(t, 0, 4, len(t), False) == (0, 11, 2, 0, 8)


@pytest.mark.gpu
def test_device_simple_scan_matches_reference(gpu_ctx, simple_golden):
    for name, case in simple_golden.items():
        _cmp(_device(name, case["seq"], case["params"], case["tier1_seen"]), case["records"])


def _seeded(n, seed, sub=0.02):
    r = np.random.default_rng(seed)
    B = np.frombuffer(b"ACGT", dtype=np.uint8)
    out = bytearray()
    while len(out) < n:
        out += B[r.integers(0, 4, int(r.integers(30, 400)))].tobytes()
        u = int(r.integers(2, 60))
        arr = bytearray(B[r.integers(0, 4, u)].tobytes() * int(r.integers(2, 12)))
        for q in range(len(arr)):
            if r.random() < sub:
                arr[q] = B[r.integers(0, 4)]
        out += arr
    return bytes(out[:n])


@pytest.mark.gpu
@pytest.mark.parametrize("n,seed,params", [(3000, 1, {}), (9000, 2, {}), (20000, 3, {}),
                                          (4000, 4, dict(allow_mismatches=False)),
                                          (150_000, 5, dict(min_period=8))])
def test_device_simple_scan_vs_oracle(gpu_ctx, n, seed, params):
    seq = _seeded(n, seed)
    want = _oracle("c", seq, params, [])
    assert want
    _cmp(_device("c", seq.decode(), params, []), want)


@pytest.mark.gpu
def test_device_simple_scan_iteration_cap(gpu_ctx):
    """2 Mbp: 6 period walks x ~20,000 positions -- the reference's global
    100,000-iteration cap ends the scan inside the fifth walk."""
    seq = _seeded(2_000_000, 9, 0.01)
    want = _oracle("c", seq, {}, [])
    _cmp(_device("c", seq.decode(), {}, []), want)
