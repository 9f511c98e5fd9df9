"""Step-by-step device bring-up with flushed progress (debug aid)."""
import os, sys, time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "bwt-algorithm_amd")]
t0 = time.time()
def log(*a):
    print(f"[{time.time()-t0:7.2f}s]", *a, flush=True)
import numpy as np
log("numpy ok")
import oracle
from bwtmi import _lib, synth
log("imports ok")
L = _lib.lib(); log("lib loaded, devices:", _lib.device_count())
h = _lib.ctx(0); log("ctx open")
_lib.kernel_stats(h, True, True)
from bwtmi.tiers import strict_scan_hits
for n in [int(x) for x in sys.argv[1:]] or [100, 1000, 20000]:
    seq = synth.generate_contig(n, 11, 0.0)
    log("scan n=", n)
    g = strict_scan_hits(np.frombuffer(seq, dtype=np.uint8), 1, max(120, min(n // 3, 1000)), 3)
    o = oracle.strict_scan(seq, 1, max(120, min(n // 3, 1000)), 0, 3)
    log("  gpu", g.shape, "oracle", o.shape, "equal", g.shape == o.shape and bool((g == o).all()))
    log("  kernels", _lib.kernel_stats(h, True, True))
from bwtmi import BWTCore
for n in [50, 5000]:
    text = synth.generate_contig(n, 3) + b"$"
    log("index n=", n)
    core = BWTCore(text.decode())
    ref = oracle.Index(text)
    log("  sa equal", bool((core.suffix_array == ref.sa).all()), "bwt equal", bool((core.bwt_arr == ref.bwt).all()))
log("done")
