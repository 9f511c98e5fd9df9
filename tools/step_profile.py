"""Per-call wall time, CPU time (all threads) and minor page faults of the bench step on the GPU box
(C3, one 100 Mbp contig).  usage: python tools/step_profile.py [steps] [contig_bp]"""
import os, resource, sys, time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "bwt-algorithm_amd")]
from bwtmi import _lib, synth
from bwtmi.records import Job

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
n = int(sys.argv[2]) if len(sys.argv) > 2 else 100_000_000
ctx = _lib.ctx(0)
threads = int(os.environ.get("STEP_THREADS", "0"))   # 0 = the library default (<= 16)
job = Job(min_copies=3, max_unit_len=120, show_progress=True, tier2=True, build_index=True, sa_sample=32,
          threads=threads)
job.add_contig("contig1", synth.generate_contig(n, 1, 0.0), 30, 30)
job.select([0])
job.upload(ctx)
out = os.path.join(os.environ.get("TMPDIR", "/tmp"), "step_profile.tab")
if os.environ.get("STEP_KSTATS") == "1":   # live per-kernel HIP-event timing, as bench.py runs it
    _lib.kernel_stats(ctx, enable=True, reset=True)
for s in range(steps):
    row = []
    for name, fn in (("reset", job.reset), ("scan", lambda: job.scan(ctx)), ("post", job.postprocess),
                     ("write", lambda: job.write("strfinder", out)), ("wait", lambda: job.wait(ctx))):
        if name == "scan":
            job.select([0])
        r0 = resource.getrusage(resource.RUSAGE_SELF)
        t = time.perf_counter(); fn(); dt = (time.perf_counter() - t) * 1e3
        r1 = resource.getrusage(resource.RUSAGE_SELF)
        cpu = (r1.ru_utime + r1.ru_stime - r0.ru_utime - r0.ru_stime) * 1e3
        row.append(f"{name} {dt:.1f}ms/cpu {cpu:.0f}ms/{r1.ru_minflt - r0.ru_minflt}pf")
    print(f"step {s}: " + "  ".join(row), " stages", [round(x, 1) for x in job.stage_ms()], flush=True)
os.unlink(out)
