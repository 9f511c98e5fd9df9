"""Host-stage CPU profile without a device: oracle strict hits fed through
bwtmi_job_add_hits, then postprocess + write, repeated under the SIGPROF
sampler (tools/libsampler.so).  usage: python tools/sampler_post.py OUT_PREFIX BP THREADS [ITERS] [SUB]"""
import ctypes, os, sys, time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "bwt-algorithm_amd"), os.path.join(REPO, "tools")]
import numpy as np
import oracle
from sampler import report
from bwtmi import synth
from bwtmi.records import Job

prefix, n, threads = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
iters = int(sys.argv[4]) if len(sys.argv) > 4 else 10
sub = float(sys.argv[5]) if len(sys.argv) > 5 else 0.0
seq = synth.generate_contig(n, 1, sub)
cache = f"/tmp/hits_{n}_{sub}.npy"
if os.path.exists(cache):
    hits = np.load(cache)
else:
    hits = oracle.strict_scan(seq[30:-30], 1, 1000, 0, 3, threads=8)
    np.save(cache, hits)
j = Job(min_copies=3, show_progress=True, threads=threads)
j.add_contig("contig1", seq, 30, 30)
out = "/tmp/sampler_post.tab"
lib = ctypes.CDLL(os.path.join(REPO, "tools", "libsampler.so"))
def it():
    j.reset(); j.add_hits(0, hits); j.postprocess(); j.write("strfinder", out)
it()
print("threads sampled:", lib.sampler_start(2000), flush=True)
t0 = time.time()
for _ in range(iters):
    it()
print(f"{(time.time() - t0) * 1e3 / iters:.1f} ms/iter", flush=True)
ns = lib.sampler_stop((prefix + ".raw").encode())
report(prefix, prefix + ".raw")
