"""Tier 3 long-read anchoring (bwt.py:2828-3036, CLI
bwt.py:3917-3924 and 4312-4328).

tests/golden/tier3.json holds the reference's own outputs (make_goldens.py
tier3): Tier3LongReadFinder.find_very_long_repeats on three seeded contigs
against 27 long reads, and CLI runs with --tier3 --long-reads (FASTA and FASTQ
reads, four formats, parallel mode, and --jobs -1 where the reference skips
Tier 3).  CPU tests pin the oracle restatement (oracle/library.py tier3,
oracle/post.py run_file) to them; GPU tests check the device path against the
goldens and against the oracle on seeded inputs."""
import dataclasses
import hashlib
import json
import os

import numpy as np
import pytest

import oracle
from oracle import library as olib
from oracle import post

FIELDS = ("start", "end", "motif", "copies", "length", "tier", "confidence", "consensus_motif",
          "mismatch_rate", "max_mismatches_per_copy", "n_copies_evaluated", "strand", "percent_matches",
          "percent_indels", "score", "composition", "entropy", "actual_sequence", "variations")


@pytest.fixture(scope="module")
def t3_golden(golden_dir):
    path = os.path.join(golden_dir, "tier3.json")
    if not os.path.exists(path):
        pytest.skip("tier3.json not generated")
    with open(path) as f:
        return json.load(f)


def _inputs(golden_dir):
    seqs, full, offs = post.load_fasta(os.path.join(golden_dir, "inputs", "tier3.fa"), 30)
    reads = post.read_long_reads(os.path.join(golden_dir, "inputs", "tier3_reads.fa"))
    return seqs, reads


def _cmp(got, want, fields=FIELDS):
    assert len(got) == len(want), (len(got), len(want))
    for g, w in zip(got, want):
        for k in fields:
            gv, wv = g[k], w[k]
            if isinstance(wv, float) or isinstance(gv, float):
                assert float(gv) == float(wv), (k, g, w)
            else:
                assert gv == wv, (k, g, w)


def _raw_reads(golden_dir):
    """The reads as the library call got them (make_goldens passes the generated
    strings, before any upper-casing): FASTA records joined line by line."""
    reads, cur = [], None
    with open(os.path.join(golden_dir, "inputs", "tier3_reads.fa")) as f:
        for line in f:
            line = line.rstrip("\n")
            if line.startswith(">"):
                if cur is not None:
                    reads.append(cur)
                cur = ""
            else:
                cur += line
    if cur is not None:
        reads.append(cur)
    return reads


# ------------------------------------------------------------------------ CPU
def test_oracle_tier3_matches_reference(golden_dir, t3_golden):
    seqs, _ = _inputs(golden_dir)
    reads = [r.encode() for r in _raw_reads(golden_dir)]
    for name, case in t3_golden["library"].items():
        got = olib.tier3((seqs[name] + "$").encode(), reads, name)
        _cmp(got, case["records"])


def test_long_read_reader_handles_fasta_and_fastq(golden_dir):
    fa = post.read_long_reads(os.path.join(golden_dir, "inputs", "tier3_reads.fa"))
    fq = post.read_long_reads(os.path.join(golden_dir, "inputs", "tier3_reads.fq"))
    raw = _raw_reads(golden_dir)
    assert fa == [r.upper() for r in raw]
    # FASTQ: the quality line is appended to the sequence (bwt.py:4324-4325)
    assert fq == [r.upper() + "I" * len(r) for r in raw[:8]]
    from bwtmi.cli import _read_long_reads
    assert _read_long_reads(os.path.join(golden_dir, "inputs", "tier3_reads.fq")) == fq


@pytest.mark.parametrize("tag", ["fa.strfinder", "fa.bed", "fa.vcf", "fa.trf_dat", "fq.strfinder"])
def test_oracle_cli_with_tier3_matches_reference(golden_dir, t3_golden, tag):
    case = t3_golden["cli"][tag]
    args = case["args"]
    fmt = args[args.index("--format") + 1] if "--format" in args else "strfinder"
    reads = post.read_long_reads(os.path.join(golden_dir, "inputs", args[args.index("--long-reads") + 1]))
    out = post.run_file(os.path.join(golden_dir, "inputs", "tier3.fa"), fmt, long_reads=reads)
    assert out == case["text"]


# ------------------------------------------------------------------------ GPU
def _dev_records(seq: str, reads, name: str):
    from bwtmi import BWTCore
    from bwtmi.tiers import Tier3LongReadFinder
    return [dataclasses.asdict(r) for r in Tier3LongReadFinder(BWTCore(seq + "$")).find_very_long_repeats(reads, name)]


@pytest.mark.gpu
def test_device_tier3_matches_reference(gpu_ctx, golden_dir, t3_golden):
    seqs, _ = _inputs(golden_dir)
    reads = _raw_reads(golden_dir)
    for name, case in t3_golden["library"].items():
        got = _dev_records(seqs[name], reads, name)
        for g in got:
            g.pop("chrom")
        _cmp(got, case["records"])


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_device_tier3_vs_oracle(gpu_ctx, seed):
    """Seeded contig with long-period arrays; reads with noise, chimeras and
    windows that straddle array ends."""
    r = np.random.default_rng(100 + seed)
    B = np.frombuffer(b"ACGT", dtype=np.uint8)
    seq = bytearray(B[r.integers(0, 4, 3000)].tobytes())
    for _ in range(6):
        u = int(r.integers(10, 170))
        unit = B[r.integers(0, 4, u)].tobytes()
        arr = bytearray(unit * int(r.integers(4, 1500 // u + 5)))
        for q in range(len(arr)):
            if r.random() < 0.015:
                arr[q] = B[r.integers(0, 4)]
        seq += arr + B[r.integers(0, 4, int(r.integers(100, 700)))].tobytes()
    seq = bytes(seq)
    reads = []
    for _ in range(40):
        a = int(r.integers(0, len(seq) - 1000))
        rd = bytearray(seq[a:a + int(r.integers(900, 4000))])
        if r.random() < 0.4:
            for q in range(len(rd)):
                if r.random() < 0.005:
                    rd[q] = B[r.integers(0, 4)]
        reads.append(rd.decode())
    want = olib.tier3(seq + b"$", [x.encode() for x in reads], "c")
    got = _dev_records(seq.decode(), reads, "c")
    assert len(want) > 5
    for g in got:
        g.pop("chrom")
    _cmp(got, want)


@pytest.mark.gpu
@pytest.mark.parametrize("tag", ["fa.strfinder", "fa.bed", "fa.vcf", "fa.trf_dat", "fq.strfinder", "fa.sequential"])
def test_device_cli_with_tier3_matches_reference(gpu_ctx, golden_dir, t3_golden, tmp_path, tag):
    import contextlib
    import io
    import shutil
    from bwtmi import cli
    case = t3_golden["cli"][tag]
    for fn in ("tier3.fa", "tier3_reads.fa", "tier3_reads.fq"):
        shutil.copy(os.path.join(golden_dir, "inputs", fn), tmp_path / fn)
    cwd = os.getcwd()
    try:
        os.chdir(tmp_path)
        with contextlib.redirect_stdout(io.StringIO()):
            cli.main(["tier3.fa", "-o", "out.tab"] + case["args"])
    finally:
        os.chdir(cwd)
    got = (tmp_path / "out.tab").read_bytes()
    assert hashlib.sha256(got).hexdigest() == case["sha256"], got.decode()[:2000]
