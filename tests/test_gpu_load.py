"""Whole-file loads with the analysed sequences built on the device
(bwtmi_job_load_fasta_dev, csrc/fasta_dev.hip) against the host loader, which
the CPU suite pins to load_reference (bwt.py:3713-3756; test_host.py):

* every golden input FASTA (edge cases: CRLF and lone CR, a literal '$',
  natural-key collisions, contigs of 0-64 bp, lower case);
* a ~25 MB file mixing plain stretches (LF only, no padding: rebuilt on the
  device) with messy ones (CR/CRLF, padded and blank lines: written on the
  host and copied up), lower case, N, duplicate names, tiny and empty contigs,
  one-base and very long lines;
* the host copies written behind the device work are complete for every
  reader (contig_seq right after the load, the scan, a reload).
Byte work: every comparison is exact."""
import glob
import os

import numpy as np
import pytest

from oracle import post

pytestmark = pytest.mark.gpu


def _check_job_pair(ctx, path, trim=30, threads=None):
    from bwtmi.records import Job
    kw = {} if threads is None else {"threads": threads}
    h = Job(**kw)
    h.load_fasta(path, trim)
    d = Job(**kw)
    d.load_fasta(path, trim, dev_ctx=ctx)
    assert d.names == h.names
    for cid in range(h.contig_count()):
        assert d.contig_info(cid) == h.contig_info(cid)
        _, fl, tl, tr = h.contig_info(cid)
        want = h.contig_seq(cid)
        assert d.contig_seq(cid) == want, h.names[cid]                  # the deferred host copy
        assert d.device_text(ctx, cid) == want[tl:fl - tr], h.names[cid]  # the device copy
    return h, d


def test_device_load_matches_host_on_golden_inputs(gpu_ctx, golden_dir):
    from bwtmi import _lib
    from bwtmi.records import Job
    paths = sorted(glob.glob(os.path.join(golden_dir, "inputs", "*.fa*")))
    assert len(paths) > 10
    failing = 0
    for p in paths:
        try:
            Job().load_fasta(p, 30)
        except _lib.BwtmiError:   # non-ASCII text: the reference fails, so does every path
            failing += 1
            with pytest.raises(_lib.BwtmiError):
                Job().load_fasta(p, 30, dev_ctx=gpu_ctx)
            continue
        seqs, full, offs = post.load_fasta(p, 30)
        h, d = _check_job_pair(gpu_ctx, p)
        for cid, nm in enumerate(d.names):
            assert d.contig_seq(cid).decode() == full[nm], (p, nm)
    assert failing >= 1


def _mixed_fasta(seed: int) -> bytes:
    r = np.random.default_rng(seed)
    eols = [b"\n", b"\r\n", b"\r"]
    out = bytearray()
    names = [f"chr{k}" for k in range(14)] + ["chr3", "tiny", "chr5"]
    for i, nm in enumerate(names):
        plain = i % 3 != 1
        out += b">" + nm.encode() + b" desc\n"
        if i % 9 == 4:
            continue                                  # empty contig
        total = 17 if nm == "tiny" else int(r.integers(200_000, 3_500_000))
        width = int(r.choice([60, 80, 1, 7, 2_500_000]))
        seq = bytes(b"ACGTacgtNn"[k] for k in r.integers(0, 10, total))
        for a in range(0, total, width):
            if plain:
                out += seq[a:a + width] + b"\n"
            else:
                pad = b" \t" if r.random() < 0.05 else b""
                out += pad + seq[a:a + width] + pad + eols[int(r.integers(3))]
                if r.random() < 0.02:
                    out += b"   " + eols[int(r.integers(3))]
    return bytes(out)


@pytest.mark.parametrize("threads", [1, 4, 16])
def test_device_load_plain_tails(gpu_ctx, tmp_path, threads):
    from test_host import _plain_tail_fasta
    path = str(tmp_path / "tails.fa")
    with open(path, "wb") as f:
        f.write(_plain_tail_fasta(threads))
    seqs, full, offs = post.load_fasta(path, 30)
    h, d = _check_job_pair(gpu_ctx, path, threads=threads)
    for cid, nm in enumerate(d.names):
        assert d.contig_seq(cid).decode() == full[nm], nm


@pytest.mark.parametrize("threads", [1, 5, 16])
def test_device_load_mixed_plain_and_messy_chunks(gpu_ctx, tmp_path, threads):
    path = str(tmp_path / "mixed.fa")
    with open(path, "wb") as f:
        f.write(_mixed_fasta(threads))
    seqs, full, offs = post.load_fasta(path, 30)
    h, d = _check_job_pair(gpu_ctx, path, threads=threads)
    assert d.names == list(seqs)
    for cid, nm in enumerate(d.names):
        assert d.contig_seq(cid).decode() == full[nm], nm


def test_device_load_scan_and_reload(gpu_ctx, tmp_path):
    """Load -> scan -> records equal the host-loaded job's; a second file
    loaded into the same job replaces the device and host copies."""
    from bwtmi import synth
    from bwtmi.records import Job
    a, b = str(tmp_path / "a.fa"), str(tmp_path / "b.fa")
    synth.write_fasta(a, [2_000_000, 700_000], 0.0)
    synth.write_fasta(b, [1_300_000], 0.02, first_index=3)
    outs = []
    for dev in (None, gpu_ctx):
        j = Job(min_copies=3, show_progress=True)
        for path in (a, b):
            j.reset()
            j.load_fasta(path, 30, dev_ctx=dev)
            j.upload(gpu_ctx)
            j.scan(gpu_ctx)
            j.postprocess()
            outs.append(j.render("strfinder"))
            j.wait(gpu_ctx)
            if dev is not None:
                for cid in range(j.contig_count()):
                    _, fl, tl, tr = j.contig_info(cid)
                    assert j.device_text(gpu_ctx, cid) == j.contig_seq(cid)[tl:fl - tr]
    assert outs[0] == outs[2] and outs[1] == outs[3]
    assert outs[0] != outs[1]


def _scan_part(job, path, world, rank, ctx=None):
    import ctypes as C
    from bwtmi._lib import check, lib
    blob, nw = C.c_void_p(), C.c_int64()
    if ctx is None:
        check(lib().bwtmi_job_fasta_scan_part(job.h, path.encode(), world, rank, C.byref(blob), C.byref(nw)))
    else:   # the part's bytes queued to ctx's device too
        check(lib().bwtmi_job_fasta_scan_part_dev(ctx, job.h, path.encode(), world, rank, C.byref(blob),
                                                  C.byref(nw)))
    try:
        return np.ctypeslib.as_array(C.cast(blob, C.POINTER(C.c_int64)), shape=(nw.value,)).copy()
    finally:
        lib().bwtmi_free(blob)


def _split_job(path, world, rank, ctx, threads, pre_ctx=None, between=None):
    """Rank `rank` of a split load, the other ranks' part tables computed here.
    pre_ctx: pass 1 also queues the part to that context's device; between():
    runs between the two passes (another load on the same context)."""
    import ctypes as C
    from bwtmi._lib import check, lib
    from bwtmi.records import Job
    parts = np.concatenate([_scan_part(Job(threads=threads), path, world, r) for r in range(world)])
    j = Job(threads=threads)
    _scan_part(j, path, world, rank, pre_ctx)   # this rank's pass-1 bytes, reused by its own contigs
    if between is not None:
        between()
    args = (j.h, path.encode(), 30, world, rank, parts.ctypes.data_as(C.c_void_p), parts.size)
    if ctx is None:
        check(lib().bwtmi_job_load_fasta_parts(*args))
    else:
        check(lib().bwtmi_job_load_fasta_parts_dev(ctx, *args))
    j.names = [j.contig_info(i)[0] for i in range(j.contig_count())]
    return j


def test_two_jobs_loaded_back_to_back_on_one_context(gpu_ctx, tmp_path):
    """Two jobs share one device context (one pinned table-staging buffer):
    the second load is queued while the first one's image upload and table
    copies may still be in flight; both jobs' device texts equal their host
    copies (the staging buffer is settled before it is rewritten)."""
    from bwtmi import synth
    from bwtmi.records import Job
    a, b = str(tmp_path / "a.fa"), str(tmp_path / "b.fa")
    synth.write_fasta(a, [40_000 + 97 * k for k in range(300)], 0.0, first_index=11)
    synth.write_fasta(b, [9_000_000, 1_500_000], 0.0, first_index=2, gaps="n2")
    jobs = []
    for path in (a, b, a):
        j = Job()
        j.load_fasta(path, 30, dev_ctx=gpu_ctx)
        jobs.append(j)
    for j in jobs:
        for cid in range(j.contig_count()):
            _, fl, tl, tr = j.contig_info(cid)
            assert j.device_text(gpu_ctx, cid) == j.contig_seq(cid)[tl:fl - tr], (j.names[cid])


@pytest.mark.parametrize("world", [2, 8])
def test_split_load_part_preloaded_on_device(gpu_ctx, tmp_path, world):
    """Pass 1 with a device queues the part's bytes to the context's FASTA image
    slot, and pass 2 on that context skips their copy when its contigs lie
    inside the part (equal contigs, one per rank) -- also when another job's
    load on the same context overwrote the slot in between (pass 2 copies
    again): the device texts equal the host split load's."""
    from bwtmi import synth
    from bwtmi.records import Job
    path = str(tmp_path / "eq.fa")
    synth.write_fasta(path, [300_000] * world, 0.0, first_index=3)
    other = str(tmp_path / "other.fa")
    synth.write_fasta(other, [200_000, 50_000], 0.0, first_index=40, gaps="n2")

    def clobber():
        Job().load_fasta(other, 30, dev_ctx=gpu_ctx)

    for rank in range(world):
        h = _split_job(path, world, rank, None, 8)
        for between in (None, clobber):
            d = _split_job(path, world, rank, gpu_ctx, 8, pre_ctx=gpu_ctx, between=between)
            assert d.names == h.names
            own = [i for i in range(h.contig_count()) if h.contig_info(i)[1] > 0]
            assert own
            for cid in own:
                _, fl, tl, tr = d.contig_info(cid)
                assert d.device_text(gpu_ctx, cid) == h.contig_seq(cid)[tl:fl - tr], (rank, cid, between)


@pytest.mark.parametrize("world", [2, 3, 8])
def test_device_split_load_matches_host(gpu_ctx, tmp_path, world):
    """The split multi-rank loader with device placement: every rank's own
    contigs on the device and on the host equal the host split load's."""
    from bwtmi import synth
    path = str(tmp_path / "split.fa")
    with open(path, "wb") as f:
        f.write(_plain_tail_fasta_mixed(world))
    for rank in range(world):
        h = _split_job(path, world, rank, None, 8)
        d = _split_job(path, world, rank, gpu_ctx, 8)
        assert d.names == h.names
        own = [i for i in range(h.contig_count()) if h.contig_info(i)[1] > 0]
        for cid in own:
            assert d.contig_info(cid) == h.contig_info(cid)
            _, fl, tl, tr = h.contig_info(cid)
            want = h.contig_seq(cid)
            assert d.contig_seq(cid) == want, (rank, h.names[cid])
            assert d.device_text(gpu_ctx, cid) == want[tl:fl - tr], (rank, h.names[cid])


def _plain_tail_fasta_mixed(seed: int) -> bytes:
    from test_host import _plain_tail_fasta
    from bwtmi import synth
    r = np.random.default_rng(seed)
    body = synth.generate_contig(3_000_000, 7)
    out = bytearray(_plain_tail_fasta(seed))
    for k in range(4):   # equal synthetic contigs, 60-column lines (the C4 shape)
        out += b">s" + str(k).encode() + b"\n"
        a = int(r.integers(0, 1_000_000))
        seq = body[a:a + 2_000_000]
        out += b"\n".join(seq[i:i + 60] for i in range(0, len(seq), 60)) + b"\n"
    return bytes(out)


_SCREEN_SCRIPT = r"""
import hashlib, os, sys
sys.path[:0] = [{repo!r}, os.path.join({repo!r}, "bwt-algorithm_amd")]
from bwtmi import _lib
from bwtmi.records import Job
ctx = _lib.ctx(0)
j = Job(min_copies=3, show_progress=True)
j.load_fasta({fa!r}, 30, dev_ctx=ctx)
j.scan(ctx)
j.postprocess()
print(hashlib.sha256(j.render("strfinder")).hexdigest(), j.count())
j.wait(ctx)
"""


def test_screened_hits_one_and_two_word_downloads(tmp_path):
    """The screened strict hits come down as one 64-bit word each when the
    longest span and motif fit (the default) or as two (BWTMI_SCREEN_WIDE=1,
    the layout of spans past 2^32 / (2 * lmax)): same records either way."""
    import subprocess
    import sys
    from bwtmi import synth
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    fa = str(tmp_path / "s.fa")
    synth.write_fasta(fa, [3_000_000, 1_000_000], 0.02)
    code = _SCREEN_SCRIPT.format(repo=repo, fa=fa)
    outs = []
    for wide in ("0", "1"):
        env = dict(os.environ, BWTMI_SCREEN_WIDE=wide)
        r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
        outs.append(r.stdout.split()[-2:])
    assert outs[0] == outs[1] and int(outs[0][1]) > 1000
