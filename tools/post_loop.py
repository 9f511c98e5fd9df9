"""Warm-loop timing of the native host stages of one contig (CPU only, no
device): oracle strict hits are fed once per iteration through
bwtmi_job_add_hits, then postprocess + render; per-stage ms of each
iteration after the first.  usage: python tools/post_loop.py BP THREADS [ITERS] [SUB_RATE]"""
import os, sys, time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "bwt-algorithm_amd")]
import numpy as np
import oracle
from bwtmi import synth
from bwtmi.records import Job

n, threads = int(sys.argv[1]), int(sys.argv[2])
iters = int(sys.argv[3]) if len(sys.argv) > 3 else 5
sub = float(sys.argv[4]) if len(sys.argv) > 4 else 0.0
seq = synth.generate_contig(n, 1, sub)
cache = f"/tmp/hits_{n}_{sub}.npy"
if os.path.exists(cache):
    hits = np.load(cache)
else:
    hits = oracle.strict_scan(seq[30:-30], 1, 1000, 0, 3, threads=8)
    np.save(cache, hits)
j = Job(min_copies=3, show_progress=True, threads=threads)
j.add_contig("contig1", seq, 30, 30)
out = "/tmp/post_loop.tab"
for it in range(iters):
    j.reset()
    j.add_hits(0, hits)
    t0 = time.perf_counter(); j.postprocess(); t1 = time.perf_counter(); j.write("strfinder", out); t2 = time.perf_counter()
    st = j.stage_ms()
    print(f"iter {it}: post {1e3*(t1-t0):.2f} ms (nested {st[2]:.2f} dedup {st[3]:.2f} merge {st[4]:.2f} "
          f"refine..filter {st[5]:.2f}) write {1e3*(t2-t1):.2f} ms (render {st[6]:.2f}) final {j.count()}", flush=True)
