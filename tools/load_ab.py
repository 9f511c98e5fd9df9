"""FASTA loader timing on the host (no GPU): the C3 file loaded repeatedly,
median ms per load.  usage: python tools/load_ab.py [bp] [reps]"""
import os, sys, tempfile, time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "bwt-algorithm_amd")]
from bwtmi import synth
from bwtmi.records import Job

bp = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 8
fa = os.path.join(tempfile.gettempdir(), "load_ab.fa")
synth.write_fasta(fa, [bp], 0.0)
j = Job()
ts = []
for _ in range(reps):
    t = time.perf_counter()
    j.reset()
    j.load_fasta(fa, 30)
    ts.append((time.perf_counter() - t) * 1e3)
print(f"plain={'off' if os.environ.get('BWTMI_NO_PLAIN') else 'on'} median {sorted(ts)[len(ts) // 2]:.2f} ms min {min(ts):.2f}")
os.unlink(fa)
