"""Wall-time split of Tier2LCPFinder.find_short_imperfect_repeats (A2-10,
bwt.py:2027-2095) on a 999 kbp seeded contig: the Python wrapper's pieces
around the C call (bwtmi_index_short_imperfect), per repetition.

usage: python tools/si_profile.py [bp] [reps]"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "bwt-algorithm_amd")]


def main():
    import ctypes as C
    import numpy as np
    from bwtmi import BWTCore, synth
    from bwtmi._lib import check, lib
    from bwtmi.records import Job
    from bwtmi.tiers import Tier2LCPFinder
    n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 999_000
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    seq = synth.generate_contig(n, 500 + n % 97, 0.02)
    core = BWTCore(seq + b"$")
    f = Tier2LCPFinder(core)
    for _ in range(reps):
        t0 = time.perf_counter()
        t = np.ascontiguousarray(core.text_arr, dtype=np.uint8)
        t1 = time.perf_counter()
        job = Job()
        job.add_contig("c", t.tobytes(), 0, 0)
        t2 = time.perf_counter()
        p = f._params()
        buf = np.zeros(2, dtype=np.int64)
        check(lib().bwtmi_index_short_imperfect(core._ctx, core._h, C.byref(p), buf.ctypes.data, 0, job.h, 0))
        t3 = time.perf_counter()
        recs = list(job.records())
        t4 = time.perf_counter()
        w0 = time.perf_counter()
        got = f.find_short_imperfect_repeats("c", set())
        w1 = time.perf_counter()
        print(f"text {1e3 * (t1 - t0):.1f} job+contig {1e3 * (t2 - t1):.1f} C call {1e3 * (t3 - t2):.1f} "
              f"records {1e3 * (t4 - t3):.1f} ms ({len(recs)}); whole call {1e3 * (w1 - w0):.1f} ms ({len(got)})",
              flush=True)


if __name__ == "__main__":
    main()
