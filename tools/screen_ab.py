"""A/B of the nested screen's segmented-kernel geometry (BWTMI_SEG_VARIANT)
on one contig: per variant the k_seg_levels / k_seg_levels_l device ms (HIP
events) and the scan call's wall ms, and the sha of the rendered output (must
not change).  usage: python tools/screen_ab.py BP [variants...]"""
import hashlib
import os
import sys
import time

sys.path[:0] = [os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bwt-algorithm_amd")]
from bwtmi import _lib, synth  # noqa: E402
from bwtmi.records import Job  # noqa: E402

bp = int(sys.argv[1])
variants = [int(v) for v in sys.argv[2:]] or [0, 1, 2, 3]
ctx = _lib.ctx(0)
_lib.bind_host(ctx)
seq = synth.generate_contig(bp, 1, 0.0)
for rep in range(2):
    for v in variants:
        if True:   # geometry variants were compared here (r05i); one geometry is kept
            j = Job(min_copies=3, show_progress=True, build_index=False)
            j.add_contig("contig1", seq, 30, 30)
            j.upload(ctx)
            j.scan(ctx)   # warm
            _lib.kernel_stats(ctx, True, True)
            walls = []
            for _ in range(3):
                t = time.perf_counter()
                j.scan(ctx)
                walls.append((time.perf_counter() - t) * 1e3)
            ks = _lib.kernel_stats(ctx, False, True)
            j.postprocess()
            sha = hashlib.sha256(j.render("strfinder")).hexdigest()[:16]
            seg = ks.get("k_seg_levels", (0, 1, 0))
            segl = ks.get("k_seg_levels_l", (0, 1, 0))
            print(f"rep {rep} variant {v}: scan wall {sorted(walls)[1]:.3f} ms  k_seg_levels {seg[0] / seg[1]:.3f} ms"
                  f"  k_seg_levels_l {segl[0] / segl[1]:.3f} ms  sha {sha}", flush=True)
