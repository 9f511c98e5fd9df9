"""The first steps of a fresh process under the device bound checks
(BWTMI_DEVICE_CHECKS=1, device.h Ctx::checks).

Round 5 saw one illegal memory access in the first warmup step of a bench run
(background index build, reported at the first host wait after the suffix
sort's first ranks).  These runs repeat exactly that step shape
-- a fresh process and context, device FASTA load, strict scan with the index
build queued behind it on a background thread while the host post-processes
and writes, kernel timers on -- with every radix ticket, scatter slot,
first-rank position, end fix-up slot and run-list / run-end bound tested on the
device: a violation is reported by name instead of faulting, and the outputs
must equal the reference-pipeline goldens."""
import hashlib
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_STEPS = r"""
import hashlib, json, os, sys
sys.path[:0] = [{repo!r}, os.path.join({repo!r}, "bwt-algorithm_amd")]
from bwtmi import _lib
from bwtmi.records import Job
assert _lib.knob("DEVICE_CHECKS") == 1
ctx = _lib.ctx(0)
_lib.bind_host(ctx)
out = {{}}
for name, fa in {files!r}:
    job = Job(min_copies=3, max_unit_len=120, show_progress=True, tier2=True, build_index=True, sa_sample=32)
    shas = []
    for step in range(3):
        if step == 1:
            _lib.kernel_stats(ctx, enable=True, reset=True)   # the bench's timed steps run with timers on
        job.reset()
        job.load_fasta(fa, 30, dev_ctx=ctx)
        job.upload(ctx)
        job.scan(ctx)
        job.postprocess()
        tab = fa + ".tab"
        job.write("strfinder", tab)
        job.wait(ctx)
        with open(tab, "rb") as f:
            shas.append(hashlib.sha256(f.read()).hexdigest())
        os.unlink(tab)
    _lib.kernel_stats(ctx, enable=False, reset=True)
    out[name] = shas
print(json.dumps(out))
"""


def test_first_steps_under_device_checks(golden_dir, tmp_path):
    from bwtmi import synth
    with open(os.path.join(golden_dir, "expected_large.json")) as f:
        goldens = json.load(f)
    files = []
    for name in ("G12N", "C4"):   # 3-bit symbol sort with N runs (deep runs); 8 ACGT contigs on the lanes
        g = goldens[name]
        fa = str(tmp_path / f"{name}.fa")
        assert synth.write_fasta(fa, g["lengths"], g["sub_rate"], g.get("first_index", 1),
                                 g.get("gaps")) == g["fasta_sha256"]
        files.append((name, fa))
    env = dict(os.environ, BWTMI_DEVICE_CHECKS="1")
    r = subprocess.run([sys.executable, "-c", _STEPS.format(repo=REPO, files=files)], env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    got = json.loads(r.stdout.strip().splitlines()[-1])
    for name, _ in files:
        assert got[name] == [goldens[name]["out_sha256"]] * 3, name


def test_device_checks_on_suffix_sorts_and_scan(gpu_ctx):
    """The suffix sorts of every class the oracle tests use (ACGT with long
    runs and shared prefixes, N runs, the general doubling) and a strict scan,
    with the bound checks on in this process: no check fires and the results
    stay the oracle's."""
    from bwtmi import _lib, synth
    from test_gpu import _check_index, _same, _planted
    with _lib.knobs(DEVICE_CHECKS=1):
        _check_index(synth.shared_prefix_runs(b"ACGT", 5) + b"$")
        _check_index(synth.generate_contig(400_000, 31, gaps="n2") + b"$")
        _check_index(synth.generate_contig(300_000, 32) + b"A" * 40 + b"$")
        _check_index(_planted(20_000, 9, b"ACGTNRYK") + b"$")
        _same(_planted(300_000, 33), 1, 1000, 3)
