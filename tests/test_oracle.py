"""Pin the CPU oracle (oracle/) against the reference's own outputs.

Every vector under tests/golden was produced by running the reference itself
(tests/golden/make_goldens.py, build container only).  The oracle is then
trusted as the checker of the HIP path at sizes the goldens do not cover.
"""
import hashlib
import json
import os

import numpy as np
import pytest

import oracle
from oracle import post


def _load(golden_dir, name):
    with open(os.path.join(golden_dir, name)) as f:
        return json.load(f)


def _cli_args(args):
    d = dict(fmt="strfinder", mc=3, trim=30, tier2=True)
    for i, a in enumerate(args):
        if a == "--format":
            d["fmt"] = args[i + 1]
        elif a == "--min-copies":
            d["mc"] = int(args[i + 1])
        elif a == "--flank-trim":
            d["trim"] = int(args[i + 1])
        elif a == "--tier1":
            d["tier2"] = False
    return d


def test_strict_scan_matches_reference_raw_hits(golden_dir):
    raw = _load(golden_dir, "rawhits.json")
    assert len(raw) > 30
    for key, case in raw.items():
        seq = case["seq"].encode()
        hits = oracle.strict_scan(seq, case.get("min_unit", 1), case["U"], case.get("max_mismatch", 0),
                                  case["min_copies"])
        got = [[int(s), int(e), seq[s:s + p].decode(), int(c)] for s, e, L, p, c in hits.tolist()]
        assert got == case["hits"], key


def test_strict_scan_known_synthetic_test_rows():
    # synthetic_test.fa yields 14 raw hits with U=27..1
    seq = open(os.path.join(os.path.dirname(__file__), "golden", "inputs",
                            "synthetic_test.fa")).read().split("\n", 1)[1].replace("\n", "")[30:-30]
    hits = oracle.strict_scan(seq.encode(), 1, 120, 0, 3)
    assert len(hits) == 14
    assert (np.diff(hits[:, 2]) <= 0).all()          # unit_len descending


def test_cli_outputs_via_python_oracle(golden_dir):
    man = _load(golden_dir, "expected_cli.json")
    for name, m in sorted(man.items()):
        d = _cli_args(m["args"])
        out = post.run_file(os.path.join(golden_dir, "inputs", m["input"]), d["fmt"], d["mc"], 120,
                            d["trim"], d["tier2"]).encode()
        assert hashlib.sha256(out).hexdigest() == m["sha256"], name


def test_index_arrays_match_reference(golden_dir):
    arrs = np.load(os.path.join(golden_dir, "index_arrays.npz"))
    meta = _load(golden_dir, "index_meta.json")
    for key, m in meta.items():
        text = arrs[key + "__text"]
        ix = oracle.Index(text.tobytes())
        assert (ix.sa == arrs[key + "__sa"]).all(), key
        assert (ix.bwt == arrs[key + "__bwt"]).all(), key
        assert (ix.lcp() == arrs[key + "__lcp"]).all(), key
        for c, v in m["C"].items():
            assert ix.C[int(c)] == v, key
        for c, v in m["totals"].items():
            assert ix.totals[int(c)] == v, key
        for c, v in m["occ"].items():
            assert ix.occ[int(c), :len(v)].tolist() == v, key
        assert {str(k): v for k, v in ix.sampled_sa.items()} == m["sampled"], key
        kh = {str(c): ix.kmer_positions(c) for c in range(1 << 16) if ix.kmer_positions(c)}
        assert kh == m["kmer_hash"], key
        for p, iv in m["backward"].items():
            assert list(ix.backward_search(p.encode())) == iv, (key, p)


def test_threaded_suffix_array_equals_serial(golden_dir):
    """The baseline's threaded prefix doubling (chunk sorts + co-rank merges +
    chunked re-rank) returns the reference's suffix array: on every golden
    text, and equal to the 1-thread sort on texts large enough to take the
    parallel path (runs, repeats, N blocks, odd thread counts)."""
    arrs = np.load(os.path.join(golden_dir, "index_arrays.npz"))
    for key in _load(golden_dir, "index_meta.json"):
        assert (oracle.Index(arrs[key + "__text"].tobytes(), threads=4).sa == arrs[key + "__sa"]).all(), key
    rng = np.random.default_rng(5)
    for n, th in [(4096, 2), (50_001, 3), (200_000, 8)]:
        t = rng.choice(np.frombuffer(b"ACGTN", np.uint8), n - 1)
        t[100:2100] = ord("A")
        t[3000:3600] = np.tile(t[2900:2906], 100)
        text = np.append(t, np.uint8(36)).tobytes()
        assert (oracle.Index(text, threads=th).sa == oracle.Index(text).sa).all(), (n, th)


def test_motif_helpers_match_reference(golden_dir):
    k = _load(golden_dir, "motif_known.json")
    for w, v in k["canonical"].items():
        assert post.min_rotation(w) == v
    for w, v in k["stranded"].items():
        assert list(post.canonical_stranded(w)) == v
    for w, v in k["revcomp"].items():
        assert post.revcomp(w) == v
    for w, v in k["entropy"].items():
        assert abs(post.entropy(w) - v) < 1e-12
    for w, v in k["period"].items():
        assert post.smallest_period(w) == v
    for w, v in k["composition"].items():
        assert post.composition(w) == v
    for l, mm, v in k["score"]:
        assert post.trf_score(l, mm) == v
    for seq, s, e, m, mc, want in k["align"]:
        got = post.align_region(seq, s, e, m, min_copies=mc)
        if want is None:
            assert got is None
            continue
        assert got["consensus"] == want["consensus"]
        assert got["copies"] == want["copies"] and got["consumed"] == want["consumed"]
        assert got["mismatch_rate"] == want["mismatch_rate"]
        assert got["variations"] == want["variations"]
