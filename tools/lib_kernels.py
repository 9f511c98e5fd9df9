"""Device timing of the north_star library kernels off the CLI path (VERDICT r2
#7): Kasai LCP (k_isa, k_kasai; bwt.py:56-95, 2108-2116), the LCP plateau scan
(k_plateau_*; 2118-2145, 2500-2560), the Hamming seed-and-extend table
(k_extend; 2027-2095, 2697-2805 -- the reference skips it above 1 Mbp),
Tier 1 (k_t1_flags; 1426-1538), Tier 3 anchoring (k_t3_windows; 2828-3036) and
the simple period scan (k_simple_extend; 2177-2498), on seeded synthetic
contigs of the given sizes.  Per call: wall ms and every kernel's HIP-event
time, launches and algorithmic bytes (KLAUNCH models) -> GB/s.

usage: python tools/lib_kernels.py OUT.json [bp ...]   (default 1e6 1e7)"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "bwt-algorithm_amd")]

import numpy as np  # noqa: E402


def main():
    out = sys.argv[1]
    sizes = [int(float(x)) for x in sys.argv[2:]] or [999_000, 10_000_000]
    from bwtmi import BWTCore, _lib, synth
    from bwtmi.tiers import Tier1STRFinder, Tier2LCPFinder, Tier3LongReadFinder
    ctx = _lib.ctx(0)
    res = dict(host=_lib.host_info(), runs=[])
    for n in sizes:
        seq = synth.generate_contig(n, 500 + n % 97, 0.02)
        text = seq + b"$"
        r = np.random.default_rng(n % 1000)
        reads = [seq[a:a + 5000].decode() for a in r.integers(0, n - 5000, 64).tolist()]
        core = BWTCore(text)
        f = Tier2LCPFinder(core)
        calls = [("lcp", lambda: core.lcp_array()),
                 ("lcp_plateaus", lambda: f._detect_lcp_plateaus(None, "c")),
                 ("tier1", lambda: Tier1STRFinder(np.frombuffer(text, dtype=np.uint8), 9).find_strs("c")),
                 ("tier3", lambda: Tier3LongReadFinder(core).find_very_long_repeats(reads, "c"))]
        if n < 1_000_000:   # bwt.py:2048: the reference returns [] above 1 Mbp (text incl. '$')
            calls.append(("short_imperfect", lambda: f.find_short_imperfect_repeats("c", set())))
            calls.append(("long_repeats", lambda: f.find_long_repeats("c", set())))
        for name, fn in calls:
            fn()   # warm (slots, code objects)
            _lib.kernel_stats(ctx, enable=True, reset=True)
            t0 = time.perf_counter()
            got = fn()
            wall = (time.perf_counter() - t0) * 1e3
            ks = _lib.kernel_stats(ctx, enable=False, reset=True)
            kern = {k: dict(ms=round(v[0], 4), launches=v[1], alg_bytes=v[2],
                            gbs=round(v[2] / (v[0] / 1e3) / 1e9, 1) if v[0] > 0 and v[2] > 0 else None)
                    for k, v in sorted(ks.items(), key=lambda kv: -kv[1][0])}
            res["runs"].append(dict(bp=n, call=name, wall_ms=round(wall, 3), records=len(got), kernels=kern))
            print(json.dumps(res["runs"][-1]), flush=True)
        core.clear()
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
