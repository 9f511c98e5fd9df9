"""Time the native host post-processing on checker hits (CPU only)."""
import os, sys, time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "bwt-algorithm_amd")]
import numpy as np
import oracle
from bwtmi import synth
from bwtmi.records import Job
n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
threads = int(sys.argv[2]) if len(sys.argv) > 2 else 0
cache = f"/tmp/hits_{n}.npy"
seq = synth.generate_contig(n, 1, 0.0)
trim = seq[30:-30]
if os.path.exists(cache):
    hits = np.load(cache)
else:
    t = time.time(); hits = oracle.strict_scan(trim, 1, 1000, 0, 3, threads=8); np.save(cache, hits)
    print(f"oracle scan {time.time()-t:.1f}s", flush=True)
print("raw hits", len(hits))
j = Job(min_copies=3, show_progress=True, threads=threads)
j.add_contig("contig1", seq, 30, 30)
t = time.time(); j.add_hits(0, hits); print(f"add_hits {time.time()-t:.2f}s")
t = time.time(); j.postprocess(); tp = time.time() - t
st = j.stage_ms()
print(f"postprocess {tp:.2f}s  nested {st[2]:.0f} dedup {st[3]:.0f} merge {st[4]:.0f} rest {st[5]:.0f} ms; final {j.count()}")
t = time.time(); out = j.render("strfinder"); nl = out.count(b"\n") - 1; print(f"render {time.time()-t:.2f}s rows {nl}")
import hashlib; print("sha", hashlib.sha256(out).hexdigest()[:16])
st = j.stage_ms()
print(f"render stage {st[6]:.0f} ms")
t = time.time(); j.reset(); print(f"reset {1000*(time.time()-t):.0f} ms")
