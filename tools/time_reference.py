#!/usr/bin/env python3
"""Time the REFERENCE itself (`bwt.py IN.fa --jobs 0 --progress`) on prefixes of
the C3 contig -- build container only (the reference never travels to the GPU
box) -- and extrapolate to the 100 Mbp workloads as BASELINE.md §3 /
SURVEY.md §8(d) prescribe (per-step constant of the strict scan x
sum_L (n - 3L) steps, plus the O(k^2) nested suppression).

usage: python tools/time_reference.py OUT.json [prefix_bp ...]   (default 10000 1000000)
"""
import contextlib
import io
import json
import os
import platform
import subprocess
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "bwt-algorithm_amd")]
REF = "/root/reference"


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


def main():
    out = sys.argv[1]
    sizes = [int(x) for x in sys.argv[2:]] or [10_000, 1_000_000]
    from bwtmi import synth
    seq = synth.generate_contig(max(sizes), 1, 0.0)     # prefixes of the C3 contig
    import numpy
    info = dict(host=platform.node(), nproc=os.cpu_count(), cpu_model=cpu_model(),
                python=platform.python_version(), numpy=numpy.__version__)
    for mod in ("numba", "pydivsufsort"):
        try:
            __import__(mod)
            info[mod] = True
        except ImportError:
            info[mod] = False
    runs = []
    for n in sizes:
        work = tempfile.mkdtemp()
        fa = os.path.join(work, "in.fa")
        with open(fa, "wb") as f:
            f.write(b">contig1\n")
            for i in range(0, n, 60):
                f.write(seq[i:i + 60] + b"\n")
        cmd = [sys.executable, os.path.join(REF, "bwt.py"), fa, "-o", os.path.join(work, "out.tab"),
               "--jobs", "0", "--progress"]
        t0 = time.time()
        r = subprocess.run(cmd, cwd=work, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
        dt = time.time() - t0
        rows = sum(1 for _ in open(os.path.join(work, "out.tab"))) - 1 if r.returncode == 0 else None
        # the worker's strict scan: sum_L (n' - 3L) steps over L = U..1, n' = n - 60 (bwt.py:1920-1999)
        m = n - 60
        U = max(120, min(m // 3, 1000))
        steps = sum(max(0, m - 3 * L) for L in range(1, min(U, m // 3) + 1))
        runs.append(dict(bp=n, seconds=round(dt, 2), rc=r.returncode, rows=rows, scan_steps=steps,
                         cmd=" ".join(cmd[1:]).replace(work, "$W")))
        print(json.dumps(runs[-1]), flush=True)
    big = runs[-1]
    # extrapolation: the larger prefix's per-step constant (it includes nested suppression
    # and post-processing), applied to the 100 Mbp scan steps; plus the O(k^2) nested term
    per_step = big["seconds"] / big["scan_steps"]
    n = 100_000_000 - 60
    steps100 = sum(n - 3 * L for L in range(1, 1001))
    k1 = 54_052 * (big["bp"] / 1e6)                   # raw hits scale with n
    k100 = k1 * 100e6 / big["bp"]
    nested_1mbp_s = 88.0                              # 85-92 s for 54k raw hits
    est = dict(per_step_us=round(per_step * 1e6, 3), scan_steps_100mbp=steps100,
               scan_seconds_100mbp=round(per_step * steps100),
               nested_seconds_100mbp=round(nested_1mbp_s * (k100 / 54_052) ** 2),
               note="C3/C5 with --progress use 1 core whatever nproc (Pool size min(cores, #contigs), "
                    "bwt.py:3863-3864); C4 uses min(cores, 8)")
    est["total_days_100mbp"] = round((est["scan_seconds_100mbp"] + est["nested_seconds_100mbp"]) / 86400, 1)
    est["mbp_per_s_100mbp"] = 100.0 / (est["scan_seconds_100mbp"] + est["nested_seconds_100mbp"])
    with open(out, "w") as f:
        json.dump(dict(info=info, runs=runs, extrapolation=est), f, indent=1)
    print(json.dumps(est))


if __name__ == "__main__":
    main()
