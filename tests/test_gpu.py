"""Parity of the HIP path (through the C ABI) with the reference goldens and
with the CPU oracle.  Integer/byte work: every comparison is exact."""
import hashlib
import json
import os

import numpy as np
import pytest

import oracle
from oracle import post

pytestmark = pytest.mark.gpu


def _rng_text(n, alphabet, seed):
    r = np.random.default_rng(seed)
    a = np.frombuffer(alphabet, dtype=np.uint8)
    return a[r.integers(0, len(a), n)].tobytes()


def _planted(n, seed, alphabet=b"ACGT", max_unit=200, density=0.3):
    """Random text with planted perfect arrays of many unit lengths."""
    r = np.random.default_rng(seed)
    t = bytearray(_rng_text(n, alphabet, seed))
    pos = 0
    while pos < n:
        pos += int(r.integers(20, 400))
        L = int(r.choice([1, 2, 3, 4, 5, 6, 7, 12, 31, 32, 33, 63, 64, 65, 100, max_unit]))
        c = int(r.integers(2, 9))
        unit = _rng_text(L, alphabet, int(r.integers(1 << 30)))
        arr = (unit * c)[: max(0, n - pos)]
        t[pos:pos + len(arr)] = arr
        pos += len(arr)
    return bytes(t)


def _gpu_hits(seq, min_unit, max_unit, mc):
    from bwtmi.tiers import strict_scan_hits
    return strict_scan_hits(np.frombuffer(seq, dtype=np.uint8), min_unit, max_unit, mc)


def _same(seq, min_unit, max_unit, mc):
    g = _gpu_hits(seq, min_unit, max_unit, mc)
    o = oracle.strict_scan(seq, min_unit, max_unit, 0, mc)
    assert g.shape == o.shape, (len(seq), max_unit, mc, g.shape, o.shape)
    assert (g == o).all(), (len(seq), max_unit, mc)
    return len(g)


# ------------------------------------------------------------------ strict scan
def test_strict_scan_reference_raw_hits(gpu_ctx, golden_dir):
    with open(os.path.join(golden_dir, "rawhits.json")) as f:
        raw = json.load(f)
    from bwtmi.tiers import strict_scan_hits
    for key, case in raw.items():   # incl. the reference's max_mismatch=2 run ("synth_imperfect.fa|mm2")
        seq = case["seq"].encode()
        h = strict_scan_hits(np.frombuffer(seq, dtype=np.uint8), case.get("min_unit", 1), case["U"],
                             case["min_copies"], max_mismatch=case.get("max_mismatch", 0))
        got = [[int(s), int(e), seq[s:s + p].decode(), int(c)] for s, e, L, p, c in h.tolist()]
        assert got == case["hits"], key


@pytest.mark.parametrize("n,alpha,seed", [
    (1, b"ACGT", 1), (2, b"A", 1), (7, b"AC", 2), (64, b"A", 3), (200, b"AT", 4), (1000, b"ACGT", 5),
    (5000, b"ACGT", 6), (5000, b"ACGTN", 7), (4000, b"ACGTNRYKM", 8), (3000, bytes(range(65, 90)), 9),
    (20000, b"ACGT", 10), (100000, b"ACGT", 11)])
def test_strict_scan_random_vs_oracle(gpu_ctx, n, alpha, seed):
    seq = _planted(n, seed, alpha) if n > 100 else _rng_text(n, alpha, seed)
    for mc in (2, 3, 4, 5):
        U = max(120, min(n // mc, 1000))
        _same(seq, 1, U, mc)
    _same(seq, 3, 40, 3)


@pytest.mark.parametrize("n,alpha,seed", [(1, b"ACGT", 1), (60, b"A", 2), (700, b"AC", 3), (5000, b"ACGT", 4),
                                          (4000, b"ACGTNRY", 5), (30000, b"ACGT", 6)])
def test_strict_scan_mismatch_vs_oracle(gpu_ctx, n, alpha, seed):
    """find_long_unit_repeats_strict with max_mismatch > 0 (bwt.py:1929-1944):
    Hamming-tolerant adjacency on the device against the oracle's direct loop."""
    from bwtmi.tiers import strict_scan_hits
    seq = _planted(n, seed, alpha) if n > 100 else _rng_text(n, alpha, seed)
    t = np.frombuffer(seq, dtype=np.uint8)
    for mm in (1, 2, 5):
        for mc, lo, hi in ((3, 1, max(120, min(n // 3, 1000))), (2, 1, 300), (1, 3, 50), (5, 20, 120)):
            g = strict_scan_hits(t, lo, hi, mc, max_mismatch=mm)
            o = oracle.strict_scan(seq, lo, hi, mm, mc)
            assert g.shape == o.shape and (g == o).all(), (n, mm, mc)


def test_strict_scan_mismatch_many_rows_vs_oracle(gpu_ctx):
    """max_mismatch > 0 with min_copies 1 and max_unit >= n: more than 65,535
    unit lengths, so the device batches its rows (gridDim.y of the Hamming
    pass is at most 65,535)."""
    from bwtmi.tiers import strict_scan_hits
    seq = _planted(80_000, 31, b"ACGTN")
    t = np.frombuffer(seq, dtype=np.uint8)
    g = strict_scan_hits(t, 1, 80_000, 1, max_mismatch=1)
    o = oracle.strict_scan(seq, 1, 80_000, 1, 1)
    assert g.shape == o.shape and (g == o).all()


def test_strict_scan_long_runs_and_streaks(gpu_ctx):
    # homopolymers and long periodic arrays: runs spanning many 32-position words
    parts = [b"A" * 5000, b"ACGT" * 700, b"G" * 33, b"CA" * 1000, _rng_text(997, b"ACGT", 3) * 4,
             b"T" * 64, b"ACG" * 22, b"N" * 300]
    seq = b"".join(parts)
    for mc in (2, 3, 6):
        _same(seq, 1, 1000, mc)


def test_strict_scan_long_units_tile_halo(gpu_ctx):
    """--max-unit-len beyond 1000: the sampled groups of unit
    lengths >= 1088 read words w + g + 1 past the LDS tile's owned words, so the
    halo after the tile is sized from the launch's largest group.  Arrays of
    unit 1050-2000 planted across tile ends (2048/B words), against the oracle."""
    r = np.random.default_rng(77)
    t = bytearray(_rng_text(400_000, b"ACGT", 77))
    pos = 500
    while pos < len(t) - 9000:
        L = int(r.integers(1050, 2001))
        unit = _rng_text(L, b"ACGT", int(r.integers(1 << 30)))
        arr = unit * int(r.integers(2, 5))
        t[pos:pos + len(arr)] = arr
        pos += len(arr) + int(r.integers(50, 3000))
    seq = bytes(t)
    for mc in (2, 3):
        assert _same(seq, 1, 2000, mc) > 0
    _same(seq, 1100, 1900, 2)
    four = _planted(150_000, 78, b"ACGTNR", max_unit=1500)   # 4 bit planes: a shorter tile
    _same(four, 1, 1500, 2)


@pytest.mark.parametrize("kv", [{"RUNS_DENSE": 1}, {"RUNS_UNTILED": 1}])
def test_strict_scan_alternate_kernels_vs_oracle(gpu_ctx, kv):
    """The strict scan's alternate paths (BWTMI_RUNS_DENSE: every group in the
    dense kernel; BWTMI_RUNS_UNTILED: sampled groups straight from the planes)
    find the same hits: planted arrays on 2- and 4-plane texts, long units
    across tile ends, homopolymers."""
    from bwtmi import _lib
    texts = [_planted(120_000, 91), _planted(60_000, 92, b"ACGTNR", max_unit=700),
             b"A" * 4000 + _rng_text(3000, b"ACGT", 93) + b"CAG" * 900]
    with _lib.knobs(**kv):
        for seq in texts:
            for mc in (2, 3, 5):
                _same(seq, 1, 1000, mc)
        _same(_planted(200_000, 94, max_unit=1700), 1, 1800, 2)


def test_strict_scan_min_copies_one(gpu_ctx):
    seq = _planted(600, 21)
    _same(seq, 1, 200, 1)


def test_strict_scan_synthetic_1mbp_vs_oracle(gpu_ctx):
    from bwtmi import synth
    for sub in (0.0, 0.02):
        seq = synth.generate_contig(1_000_000, 40, sub)
        assert _same(seq, 1, 1000, 3) > 1000


def test_strict_scan_10mbp_with_gaps_vs_oracle(gpu_ctx):
    """A 10 Mbp contig with assembly gaps (4.1 % N in runs of 10 bp - 289 kbp,
    ~1000 single R/Y; GAP_PROFILES "n2"): raw-byte compares with N == N
    (bwt.py:1941), so every N run yields one hit per unit length; the text's
    six symbols take the 4-plane scan.  Against the oracle, bit-exact."""
    from bwtmi import synth
    seq = synth.generate_contig(10_000_000, 2, gaps="n2")
    assert _same(seq, 1, 1000, 3) > 10000


# ------------------------------------------------------------------ CLI end to end
def _cli(args):
    d = dict(fmt="strfinder", mc=3, trim=30, tier2=True)
    for i, x in enumerate(args):
        if x == "--format":
            d["fmt"] = args[i + 1]
        elif x == "--min-copies":
            d["mc"] = int(args[i + 1])
        elif x == "--flank-trim":
            d["trim"] = int(args[i + 1])
        elif x == "--tier1":
            d["tier2"] = False
    return d


def test_cli_outputs_match_reference_goldens(gpu_ctx, golden_dir, tmp_path):
    from bwtmi import TandemRepeatFinder
    with open(os.path.join(golden_dir, "expected_cli.json")) as f:
        man = json.load(f)
    for name, m in sorted(man.items()):
        d = _cli(m["args"])
        f = TandemRepeatFinder(os.path.join(golden_dir, "inputs", m["input"]), min_copies=d["mc"],
                               flank_trim=d["trim"])
        f.load_reference()
        reps = f.find_tandem_repeats_parallel(True, d["tier2"], False, None)
        out = tmp_path / f"{name}.out"
        f.save_results(reps, str(out), d["fmt"])
        assert hashlib.sha256(out.read_bytes()).hexdigest() == m["sha256"], name


def test_cli_entry_point(gpu_ctx, golden_dir, tmp_path):
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    bwt = os.path.join(here, "..", "bwt-algorithm_amd", "bwt.py")
    out = tmp_path / "repeat.tab"
    subprocess.run([sys.executable, bwt, os.path.join(golden_dir, "inputs", "test.fa"), "-o", str(out),
                    "--jobs", "0"], check=True, capture_output=True)
    with open(os.path.join(golden_dir, "expected_cli.json")) as f:
        want = json.load(f)["test.fa.strfinder"]["sha256"]
    assert hashlib.sha256(out.read_bytes()).hexdigest() == want


def test_reference_unittest_on_device(gpu_ctx, golden_dir):
    """The reference's tests/test_repeat_outputs.py, through the device path."""
    from bwtmi import TandemRepeatFinder
    f = TandemRepeatFinder(os.path.join(golden_dir, "inputs", "test2.fa"), show_progress=False,
                           max_motif_length=12)
    f.build_indices(f.load_reference())
    reps = f.find_tandem_repeats(enable_tier1=True, enable_tier2=True, enable_tier3=False)
    by = {}
    for r in reps:
        by.setdefault(r.chrom, []).append(r)
    (r1,) = by["test1_PERFECT_7mer_5copies"]
    assert (r1.start, r1.end, r1.motif, r1.variations) == (30, 65, "TCATCGG", None)
    (r4,) = by["test4_INTERRUPTED_7mer_11copies"]
    assert set(r4.variations) == {"6:5:C>A", "10:6:G>A", "11:0:ins(G)"}
    motifs = {r.motif for r in by["test6_NESTED_long20_short4"]}
    assert {"TGCTGATCGTAGCTAGCTGA", "TGCT"} <= motifs and "CTGA" not in motifs
    (r12,) = by["test12_LONG_IMPERFECT_indel"]
    assert any(v.startswith("9:10:del(") for v in r12.variations)


def test_pipeline_seeded_imperfect_vs_oracle(gpu_ctx, tmp_path):
    from bwtmi import TandemRepeatFinder, synth
    fa = str(tmp_path / "imp.fa")
    synth.write_fasta(fa, [60000, 25000], 0.03, first_index=900)
    for fmt in ("strfinder", "vcf", "trf_table"):
        f = TandemRepeatFinder(fa)
        f.load_reference()
        reps = f.find_tandem_repeats_parallel()
        out = tmp_path / "o.tab"
        f.save_results(reps, str(out), fmt)
        assert out.read_text() == post.run_file(fa, fmt), fmt


def _job_output(contigs, screen: bool, mc=3, fmt="strfinder"):
    """Scan + post-process + render through the job API; screen selects the
    device (nested.hip) or the host nested/sort/dedup stage."""
    from bwtmi import _lib
    from bwtmi.records import Job
    with _lib.knobs(HOST_SCREEN=0 if screen else 1):
        j = Job(min_copies=mc, show_progress=True)
        for name, seq in contigs:
            j.add_contig(name, seq, 30 if len(seq) > 60 else 0, 30 if len(seq) > 60 else 0)
        j.scan(_lib.ctx())
        raw = j.raw_count()
        j.postprocess()
        return raw, j.render(fmt)


@pytest.mark.parametrize("case", ["planted", "synthetic", "imperfect", "same_unit", "tiny"])
def test_device_screen_matches_host(gpu_ctx, case):
    """nested suppression + sort + dedup on the device == the host restatement,
    for the segmented single-launch screen and the per-level launches
    (BWTMI_SEG_LEVELS=0)."""
    from bwtmi import _lib
    from bwtmi import synth
    if case == "planted":
        contigs = [("p1", _planted(300_000, 5, max_unit=400, density=0.5)), ("p2", _planted(50_000, 6))]
    elif case == "synthetic":
        contigs = [("contig1", synth.generate_contig(2_000_000, 1, 0.0))]
    elif case == "imperfect":
        contigs = [("c7", synth.generate_contig(1_000_000, 7, 0.02))]
    elif case == "same_unit":   # equal natural keys -> one fold unit over two contigs
        contigs = [("chr01", _planted(40_000, 8)), ("CHR1", _planted(40_000, 9)), ("chr2", _planted(9_000, 10))]
    else:
        contigs = [("a", b"ACACACACAC"), ("b", b"A" * 7), ("c", b"")]
    for fmt in ("strfinder", "bed"):
        rd, d = _job_output(contigs, True, fmt=fmt)
        rh, h = _job_output(contigs, False, fmt=fmt)
        assert rd == rh
        assert d == h, (case, fmt)
    with _lib.knobs(SEG_LEVELS=0):
        assert _job_output(contigs, True, fmt="strfinder")[1] == _job_output(contigs, False, fmt="strfinder")[1]


@pytest.mark.parametrize("mc", [1, 2, 4, 7])
def test_screen_drop_matches_host(gpu_ctx, mc):
    """The screen drops kept hits that fail the final filter and that no merge,
    refine or collapse can reach (nested.hip k_drop_flags): the job's output
    equals the host screen's (which keeps every hit) and the device screen's
    with BWTMI_SCREEN_DROP=0, for other min_copies, imperfect arrays, N gaps and
    a fold unit of several contigs; the drop removes hits."""
    from bwtmi import _lib, synth
    contigs = [("c1", synth.generate_contig(1_500_000, 20 + mc, 0.02)),
               ("c2", synth.generate_contig(600_000, 30 + mc, 0.0, gaps="n1")),
               ("p3", _planted(200_000, 40 + mc, b"ACGTN", max_unit=300, density=0.6))]
    unit = [("chr01", _planted(60_000, 50 + mc)), ("CHR1", synth.generate_contig(80_000, 60 + mc, 0.03))]
    for cs in (contigs, unit):
        for fmt in ("strfinder", "vcf"):
            rh, h = _job_output(cs, False, mc=mc, fmt=fmt)
            rd, d = _job_output(cs, True, mc=mc, fmt=fmt)
            with _lib.knobs(SCREEN_DROP=0):
                rk, k = _job_output(cs, True, mc=mc, fmt=fmt)
            assert rd == rh == rk
            assert d == h == k, (mc, fmt)


def test_screened_hits_landing_in_pieces(gpu_ctx):
    """The scan returns while its screened-hit download is still landing (in
    pieces, an event behind each; nested.hip).  A job reset or a rescan right
    after the scan waits for it before the host buffer goes, and the
    post-processing reads each piece only after it has landed: the output
    equals the host screen's whatever happens in between."""
    from bwtmi import _lib, synth
    from bwtmi.records import Job
    seq = synth.generate_contig(3_000_000, 11, 0.0)   # ~40 k kept hits: several pieces
    want = _job_output([("contig1", seq)], False)[1]
    j = Job(min_copies=3, show_progress=True)
    j.add_contig("contig1", seq, 30, 30)
    ctx = _lib.ctx()
    j.scan(ctx)
    j.reset()          # drops the landing buffer at once
    j.scan(ctx)
    j.scan(ctx)        # the second scan replaces a buffer still landing
    j.postprocess()
    assert j.render("strfinder") == want
    del j              # a job freed right after its scan
    j2 = Job(min_copies=3, show_progress=True)
    j2.add_contig("contig1", seq, 30, 30)
    j2.scan(ctx)
    del j2


def test_failing_contig_yields_error_and_no_records(gpu_ctx, golden_dir, tmp_path, capsys, monkeypatch):
    """The worker's failure convention (bwt.py:3137-3141): a contig whose device
    work fails is reported as `ERROR processing chromosome NAME: ...` and
    contributes no records; the other contigs are unaffected (the expected
    file is the oracle pipeline with that contig's strict hits removed)."""
    from bwtmi import cli
    fa = os.path.join(golden_dir, "inputs", "test2.fa")
    seqs, _, _ = post.load_fasta(fa, 30)
    victim = sorted(seqs)[3]
    monkeypatch.setenv("BWTMI_FAIL_CONTIG", victim)
    out = tmp_path / "out.tab"
    assert cli.main([fa, "-o", str(out), "--jobs", "-1"]) == 0
    assert f"ERROR processing chromosome {victim}:" in capsys.readouterr().out
    vseq = seqs[victim].encode()

    def scan(b, U, mc):
        return oracle.strict_scan(b, 1, U, 0, mc)[:0] if b == vseq else oracle.strict_scan(b, 1, U, 0, mc)
    assert out.read_text() == post.run_file(fa, "strfinder", strict_scan=scan)


def _edge_goldens():
    here = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "expected_edge.json")
    with open(here) as f:
        return json.load(f)


@pytest.mark.parametrize("name", sorted(_edge_goldens()))
def test_edge_inputs_on_device(gpu_ctx, golden_dir, tmp_path, name):
    """The drop-in CLI on the edge inputs against the
    reference CLI's outputs -- or its failure, for non-ASCII text: no output
    file and an error."""
    import shutil
    from bwtmi import cli
    m = _edge_goldens()[name]
    fa = tmp_path / m["input"]
    shutil.copy(os.path.join(golden_dir, "inputs", m["input"]), fa)
    out = tmp_path / "out.tab"
    if "error" in m:
        with pytest.raises(Exception, match="non-ASCII"):
            cli.main([str(fa), "-o", str(out), "--jobs", "-1"] + m["args"])
        assert not out.exists()
        return
    assert cli.main([str(fa), "-o", str(out), "--jobs", "-1"] + m["args"]) == 0
    assert hashlib.sha256(out.read_bytes()).hexdigest() == m["sha256"], name


def _large_goldens():
    here = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "expected_large.json")
    with open(here) as f:
        return json.load(f)


@pytest.mark.parametrize("name", sorted(_large_goldens()))
def test_full_size_goldens(gpu_ctx, golden_dir, tmp_path, name):
    """BASELINE configs at full size -- C2 (1 Mbp --tier1), C3 (100 Mbp
    --progress), C4 (8 x 12.5 Mbp), C5 (100 Mbp with 0.02 substitutions inside
    the planted arrays, --progress, default and --no-mismatches arms), and the
    general alphabet: G12N (12.5 Mbp with assembly gaps: 3.6 % N in runs up to
    289 kbp, ~1200 single R/Y) and C3Np (C3N, 100 Mbp, 3.8 % N in runs up to
    958 kbp, --progress) -- run
    through the drop-in CLI (`bwt.py IN.fa -o OUT --jobs -1 ARGS`, bwt.py:4201-4370)
    against repeat.tab hashes of the reference pipeline
    (tests/golden/make_goldens.py hybrid; strict scan and nested suppression
    restated, everything else the reference's own code)."""
    from bwtmi import cli, synth
    g = _large_goldens()[name]
    fa = str(tmp_path / f"{name}.fa")
    assert synth.write_fasta(fa, g["lengths"], g["sub_rate"], g.get("first_index", 1),
                             g.get("gaps")) == g["fasta_sha256"], name
    out = tmp_path / f"{name}.tab"
    assert cli.main([fa, "-o", str(out), "--jobs", "-1"] + list(g["args"])) == 0
    data = out.read_bytes()
    assert data.count(b"\n") - 1 == g["out_rows"], name
    assert hashlib.sha256(data).hexdigest() == g["out_sha256"], name
    os.unlink(fa)


# ------------------------------------------------------------------ FM index
def _check_index(text: bytes, golden=None):
    from bwtmi import BWTCore
    core = BWTCore(text.decode("latin-1"))
    ref = oracle.Index(text) if golden is None else None
    sa = core.suffix_array
    if golden is not None:
        assert (sa == golden["sa"]).all() and (core.bwt_arr == golden["bwt"]).all()
        assert (core.lcp_array() == golden["lcp"]).all()
        return core
    assert (sa == ref.sa).all()
    assert (core.bwt_arr == ref.bwt).all()
    for c in ref.alphabet():
        assert (core.occ_checkpoints[c] == ref.occ[c, :len(core.occ_checkpoints[c])]).all()
        assert core.char_counts[chr(c)] == ref.C[c] and core.char_totals[chr(c)] == ref.totals[c]
    assert core.sampled_sa == ref.sampled_sa
    off, pos = core.kmer_csr()
    assert (off == ref.kmer_offsets).all() and (pos == ref.kmer_pos).all()
    assert (core.lcp_array() == ref.lcp()).all()
    return core


def test_index_matches_reference_goldens(gpu_ctx, golden_dir):
    arrs = np.load(os.path.join(golden_dir, "index_arrays.npz"))
    with open(os.path.join(golden_dir, "index_meta.json")) as f:
        meta = json.load(f)
    from bwtmi import BWTCore
    for key, m in meta.items():
        text = arrs[key + "__text"].tobytes()
        core = _check_index(text, dict(sa=arrs[key + "__sa"], bwt=arrs[key + "__bwt"],
                                       lcp=arrs[key + "__lcp"]))
        for c, v in m["occ"].items():
            assert core.occ_checkpoints[int(c)].tolist() == v, key
        assert {str(k): v for k, v in core.sampled_sa.items()} == m["sampled"], key
        assert {str(k): v for k, v in core.kmer_hash.items()} == m["kmer_hash"], key
        for p, iv in m["backward"].items():
            assert list(core.backward_search(p)) == iv, (key, p)
        for p, pos in m["locate"].items():
            assert core.locate_positions(p) == pos, (key, p)
        for p, pos in m["kmer_positions"].items():
            assert core.get_kmer_positions(p) == pos, (key, p)


@pytest.mark.parametrize("n,alpha,seed", [(2, b"A", 1), (100, b"ACGT", 2), (5000, b"ACGT", 3),
                                          (3000, b"ACGTN", 4), (2000, b"acgtNRY$", 5),
                                          (200000, b"ACGT", 6)])
def test_index_vs_oracle(gpu_ctx, n, alpha, seed):
    body = _planted(n, seed, alpha) if n > 200 else _rng_text(n, alpha, seed)
    _check_index(body + b"$")


def test_index_repetitive_text(gpu_ctx):
    _check_index(b"A" * 3000 + b"$")
    _check_index((b"ACGTTGCA" * 500) + b"$")
    _check_index(b"CA" * 2000 + b"C" + b"$")


@pytest.mark.parametrize("case", ["tiny", "edges", "groups", "long_lcp", "many_arrays", "homopolymer_peel",
                                  "arrays_300k", "arrays_300k_small_lists"])
def test_dna_suffix_sort_vs_oracle(gpu_ctx, monkeypatch, case):
    """The ACGT* '$' string sort (sa_dna.hip) against the oracle's prefix
    doubling: texts built to hit every group class -- pairs (thread sort),
    tens to a thousand members (workgroup bitonic sort), many short arrays
    sharing a 16-mer (radix refinement rounds), long common prefixes, and
    suffixes running into the end inside a tied key.  The 300 kbp texts take
    the partitioned first-rank writes (>= 2^16 bases) and fill every shard of
    the next-round lists past one chunk; with the lists capped
    (BWTMI_LS_CAP) the sort gives up and the general doubling must agree."""
    r = np.random.default_rng(sum(map(ord, case)))
    B = np.frombuffer(b"ACGT", dtype=np.uint8)

    def rnd(k):
        return B[r.integers(0, 4, k)].tobytes()
    if case == "tiny":
        for t in (b"A", b"C", b"AC", b"CA", b"AAAA", b"ACGTACGT", b"TTTTTTTTTTTTTTTTTAAAA"):
            _check_index(t + b"$")
        return
    if case == "edges":      # the last 16 suffixes tie with A-padded keys of inner ones
        t = rnd(500) + b"A" * 40 + rnd(30) + b"AC" + b"A" * 14
    elif case == "groups":   # random duplicated 16-40-mers: groups of 2..60 members
        parts = []
        for _ in range(300):
            w = rnd(int(r.integers(16, 40)))
            parts += [w + rnd(int(r.integers(1, 30))) for _ in range(int(r.integers(2, 60)))]
        t = b"".join(parts)
    elif case == "long_lcp":  # long tandem arrays: groups with thousands of equal bases
        t = rnd(200) + rnd(120) * 30 + rnd(300) + rnd(7) * 400 + rnd(50) + rnd(97) * 25 + rnd(100)
    elif case == "many_arrays":   # > 1024 arrays of the same short units: refinement rounds
        parts = []
        for _ in range(3000):
            parts.append(rnd(int(r.integers(5, 40))))
            parts.append([b"AC", b"G", b"CAG", b"TTA"][int(r.integers(0, 4))] * int(r.integers(6, 30)))
        t = b"".join(parts)
    elif case.startswith("arrays_300k"):
        parts = []
        for _ in range(12000):
            parts.append(rnd(int(r.integers(3, 20))))
            parts.append([b"AC", b"G", b"CAG", b"TTA", b"GATC"][int(r.integers(0, 5))] * int(r.integers(3, 12)))
        t = b"".join(parts)
        assert len(t) > 1 << 16
    else:   # one base repeated: a large group that loses 16 suffixes per round
        t = rnd(300) + b"G" * 2500 + rnd(300)
    from bwtmi import _lib
    with _lib.knobs(LS_CAP=3000 if case.endswith("small_lists") else -1):
        _check_index(t + b"$")


@pytest.mark.parametrize("case", ["gaps_300k", "n_only", "n_edges", "seven_symbols", "long_n_run", "groups_with_n",
                                  "eight_symbols", "byte_below_dollar", "lower_case"])
def test_small_alphabet_suffix_sort_vs_oracle(gpu_ctx, case):
    """The string sort over 3-bit symbol codes (sa_dna.hip, up to 7 symbols
    above '$': ACGT with N runs and IUPAC codes; raw byte order, N between G
    and T, bwt.py:212-264) against the oracle: assembly gaps, an N-only text,
    N runs tying with the end's zero-padded keys, all seven symbols, a 70 kbp
    N run (one group losing h suffixes per doubling round), duplicated
    N-bearing k-mers; and the texts it must leave to the general doubling
    (eight symbols, a byte below '$') -- every one bit-exact."""
    from bwtmi import synth
    r = np.random.default_rng(sum(map(ord, case)))

    def rnd(k, alpha=b"ACGT"):
        a = np.frombuffer(alpha, dtype=np.uint8)
        return a[r.integers(0, len(a), k)].tobytes()
    if case == "gaps_300k":
        t = synth.generate_contig(300_000, 14, gaps="n2")
    elif case == "n_only":
        t = b"N" * 5000
    elif case == "n_edges":
        t = rnd(500, b"ACGTN") + b"N" * 40 + rnd(30) + b"NA" + b"N" * 14
    elif case == "seven_symbols":
        t = b"".join(rnd(int(r.integers(3, 30)), b"ACGTNRY") + rnd(3, b"ACGTNRY") * int(r.integers(3, 20))
                     for _ in range(2000))
    elif case == "long_n_run":
        t = rnd(3000) + b"N" * 70_000 + rnd(3000) + b"N" * 17 + rnd(40)
    elif case == "groups_with_n":
        parts = []
        for _ in range(300):
            w = rnd(int(r.integers(16, 40)), b"ACGTN")
            parts += [w + rnd(int(r.integers(1, 30)), b"ACGTN") for _ in range(int(r.integers(2, 60)))]
        t = b"".join(parts)
    elif case == "eight_symbols":
        t = _planted(20_000, 9, b"ACGTNRYK")
    elif case == "byte_below_dollar":
        t = _planted(20_000, 10, b"ACGT!")
    else:
        t = _planted(20_000, 11, b"acgtN")
    _check_index(t + b"$")


@pytest.mark.parametrize("alpha", [b"ACGT", b"ACGTNRY"])
def test_long_runs_ordered_in_closed_form_vs_oracle(gpu_ctx, alpha):
    """Suffixes inside runs of >= 16 equal symbols (sa_dna.hip Deep: first round
    by (next symbol above / below the run's, +-remaining run), later rounds by
    the rank of the run's end): runs of every symbol and of lengths 15-17, 31-33
    and up to 40 kbp, followed by smaller and larger symbols, back to back,
    at the start, running into '$', and many runs of equal length (ties broken
    by what follows them) -- against the oracle."""
    r = np.random.default_rng(len(alpha))

    def rnd(k):
        a = np.frombuffer(alpha, dtype=np.uint8)
        return a[r.integers(0, len(a), k)].tobytes()
    parts = [alpha[:1] * 40]   # a run at the start
    for i in range(600):
        c = alpha[int(r.integers(0, len(alpha)))]
        ln = int(r.choice([15, 16, 17, 31, 32, 33, 48, 64, 100, 257, 1000]))
        parts.append(bytes([c]) * ln + rnd(int(r.integers(0, 6))))
    parts.append(b"".join(bytes([alpha[k % len(alpha)]]) * 20 for k in range(50)))   # runs back to back
    parts.append(rnd(50) + bytes([alpha[-1]]) * 40_000 + rnd(30))
    for k in range(40):   # equal runs, ties broken by the following text
        parts.append(bytes([alpha[0]]) * 37 + rnd(25))
    t = b"".join(parts) + bytes([alpha[1]]) * 50    # a run into '$'
    _check_index(t + b"$")
    _check_index(bytes([alpha[0]]) * 5000 + b"$")
    _check_index(bytes([alpha[2]]) * 17 + bytes([alpha[0]]) * 33 + b"$")


@pytest.mark.parametrize("alpha", [b"ACGT", b"ACGTNRY"])
def test_runs_after_shared_prefixes_vs_oracle(gpu_ctx, alpha):
    """Repeated 16-64-symbol prefixes followed by equal runs of 16-100 symbols
    and different next symbols on the same side of the run's symbol
    (bwtmi.synth.shared_prefix_runs): Z c^r x W.  The run's closed-form rank
    must never stand for more symbols than a doubling round claims -- with
    r < 2h a (b, r) group holds suffixes that differ inside the 2h-prefix, and
    a suffix Z... reading it through rank[a + h] would tie with its twin and
    skip x (sa_dna.hip ls_key).  Against the oracle; the 1 Mbp copy
    takes the partitioned first ranks and the segmented refinement rounds."""
    from bwtmi import synth
    _check_index(synth.shared_prefix_runs(alpha, 1) + b"$")
    _check_index(synth.shared_prefix_runs(alpha, 2, run_lengths=(16, 17, 20, 31, 32, 33),
                                          prefix_lengths=(32, 64)) * 3 + b"$")
    big = b"".join(synth.shared_prefix_runs(alpha, s, run_lengths=(16, 24, 31, 40, 63), prefix_lengths=(32, 64))
                   for s in range(3, 40))
    _check_index(big[:1_000_000] + b"$")


@pytest.mark.parametrize("S", [1, 3, 16])
def test_radix_histogram_geometries(gpu_ctx, S):
    """The single-pass radix histogram with 1, 3 or 16 scatter tiles per
    workgroup (BWTMI_HIST_S; look-back chains of different lengths, partial
    last workgroups): the candidate sorts of the strict scan and the suffix
    sorts give the oracle's results."""
    from bwtmi import _lib, synth
    with _lib.knobs(HIST_S=S):
        _same(_planted(300_000, 95 + S), 1, 1000, 3)
        _check_index(synth.generate_contig(400_000, 96 + S, gaps="n1") + b"$")
        _check_index(synth.generate_contig(300_000, 99 + S) + b"$")


def test_small_alphabet_texts_through_general_doubling(gpu_ctx):
    """BWTMI_SA_SMALL=0: gap texts take the general prefix doubling (index.hip)
    instead of the 3-bit string sort; the same arrays as the oracle."""
    from bwtmi import _lib, synth
    with _lib.knobs(SA_SMALL=0):
        _check_index(synth.generate_contig(200_000, 15, gaps="n2") + b"$")
        _check_index(_planted(20_000, 16, b"ACGTNRY") + b"$")


@pytest.mark.parametrize("rank", ["packed", "bytes"])
def test_backward_search_all_short_motifs(gpu_ctx, rank):
    """Both rank structures: the packed 2-bit blocks of ACGT texts (k_bsearch2)
    and the byte BWT + sampled Occ (k_bsearch, BWTMI_FM_BYTES=1)."""
    from bwtmi import BWTCore, MotifUtils, _lib, synth
    text = synth.generate_contig(50000, 77) + b"$"
    core = BWTCore(text.decode())
    ref = oracle.Index(text)
    pats = [m for k in range(1, 7) for m in MotifUtils.enumerate_motifs(k)]
    pats += ["ACGTACGTAC", "N", "", "TTTTTTTTTT", "GATTACA", "$", "A$", "$A", "C$", text[-9:].decode(),
             text[:12].decode(), text[100:164].decode(), "ACGN"]
    with _lib.knobs(FM_BYTES=int(rank == "bytes")):
        got = core.backward_search_batch(pats)
    for p, (sp, ep) in zip(pats, got.tolist()):
        assert (sp, ep) == ref.backward_search(p.encode()), p


def test_backward_search_all_motifs_1_to_10(gpu_ctx):
    """The north_star's FM query set: every canonical primitive ACGT motif of
    length 1..10 (MotifUtils.enumerate_motifs, bwt.py:1369-1381; 145,338
    patterns) on a 1 Mbp contig, interval for interval against the oracle."""
    from bwtmi import BWTCore, MotifUtils, synth
    text = synth.generate_contig(1_000_000, 5) + b"$"
    core = BWTCore(text.decode())
    ref = oracle.Index(text)
    pats = [m for k in range(1, 11) for m in MotifUtils.enumerate_motifs(k)]
    assert len(pats) == 145338
    got = core.backward_search_batch(pats)
    for p, (sp, ep) in zip(pats, got.tolist()):
        assert (sp, ep) == ref.backward_search(p.encode()), p


def test_index_12mbp_properties(gpu_ctx):
    """C4-size contig: SA is a permutation, adjacent suffixes ascend, BWT/occ consistent."""
    from bwtmi import BWTCore, synth
    text = synth.generate_contig(12_500_000, 3) + b"$"
    core = BWTCore(text.decode())
    sa = core.suffix_array.astype(np.int64)
    n = len(text)
    assert np.array_equal(np.sort(sa), np.arange(n))
    assert sa[0] == n - 1
    r = np.random.default_rng(0)
    t = np.frombuffer(text, dtype=np.uint8)
    for k in r.integers(1, n, 3000).tolist():
        a, b = sa[k - 1], sa[k]
        assert text[a:a + 4000] <= text[b:b + 4000], k
    bwt = core.bwt_arr
    assert (bwt == t[(sa - 1) % n]).all()
    occ = core.occ_checkpoints
    for c in (65, 67, 71, 84):
        assert occ[c][-1] == int((t == c).sum())
    off, pos = core.kmer_csr()
    assert off[-1] == n - 8


def test_kernel_stats_filter(gpu_ctx):
    """bwtmi_kernel_stats_filter: with a name set only those launches are timed
    (bench.py's timed steps time only the dominant kernel), with "" every one;
    the scan's results do not depend on it."""
    from bwtmi import _lib
    seq = _planted(200_000, 123)
    ctx = _lib.ctx()
    want = _gpu_hits(seq, 1, 1000, 3)
    try:
        _lib.kernel_stats_filter(ctx, "k_runs")
        _lib.kernel_stats(ctx, enable=True, reset=True)
        got = _gpu_hits(seq, 1, 1000, 3)
        only = _lib.kernel_stats(ctx, enable=False, reset=True)
        assert set(only) == {"k_runs"} and only["k_runs"][1] >= 1
        assert got.shape == want.shape and (got == want).all()
        _lib.kernel_stats_filter(ctx, "")
        _lib.kernel_stats(ctx, enable=True, reset=True)
        _gpu_hits(seq, 1, 1000, 3)
        every = _lib.kernel_stats(ctx, enable=False, reset=True)
        assert "k_runs" in every and len(every) > 3
    finally:
        _lib.kernel_stats_filter(ctx, "")
        _lib.kernel_stats(ctx, enable=False, reset=True)
