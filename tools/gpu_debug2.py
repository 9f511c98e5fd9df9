import os, sys, time, faulthandler
faulthandler.dump_traceback_later(100, exit=True)
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "bwt-algorithm_amd")]
t0 = time.time()
def log(*a):
    print(f"[{time.time()-t0:7.2f}s]", *a, flush=True)
import numpy as np
import oracle
from bwtmi import _lib, synth, BWTCore, TandemRepeatFinder
from bwtmi.records import Job
h = _lib.ctx(0); log("ctx")
seq = synth.generate_contig(20000, 11, 0.0)
text = seq[:5000] + b"$"
log("index smoke text")
core = BWTCore(text.decode()); log("built")
ref = oracle.Index(text); log("oracle built")
log("sa eq", bool((core.suffix_array == ref.sa).all()))
g = os.path.join(REPO, "tests", "golden", "inputs", "synthetic_test.fa")
j = Job(); j.load_fasta(g, 30); log("loaded", j.names)
j.scan(h); log("scanned raw", j.raw_count())
j.postprocess(); log("post", j.count())
out = j.render("strfinder"); log("render", len(out))
f = TandemRepeatFinder(g); f.load_reference(); log("finder loaded")
r = f.find_tandem_repeats_parallel(); log("finder ran", len(r))
log("done")
