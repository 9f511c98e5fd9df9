"""Host post-processing profile without a GPU: oracle strict hits of a synthetic
contig fed through bwtmi_job_add_hits, then postprocess + write under the
sampler (tools/libsampler.so).  usage: python tools/post_profile_cpu.py PREFIX [bp] [steps]"""
import ctypes, os, sys, tempfile, time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "bwt-algorithm_amd"), os.path.join(REPO, "tools")]


def main():
    prefix = sys.argv[1]
    bp = int(sys.argv[2]) if len(sys.argv) > 2 else 20_000_000
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    import oracle
    import sampler
    from bwtmi import synth
    from bwtmi.records import Job
    seq = synth.generate_contig(bp, 1, float(os.environ.get("SUB", "0")))
    trimmed = seq[30:len(seq) - 30]
    hits = oracle.strict_scan(trimmed, 1, max(120, min(len(trimmed) // 3, 1000)), 0, 3)
    out = os.path.join(tempfile.gettempdir(), "post_profile.tab")

    def step():
        job = Job(min_copies=3, show_progress=True)
        job.add_contig("contig1", seq, 30, 30)
        job.add_hits(0, hits)
        t = time.perf_counter()
        job.postprocess()
        t1 = time.perf_counter()
        job.write("strfinder", out)
        return (t1 - t) * 1e3, (time.perf_counter() - t1) * 1e3
    step()
    lib = ctypes.CDLL(os.path.join(REPO, "tools", "libsampler.so"))
    lib.sampler_start(2000)
    ts = [step() for _ in range(steps)]
    raw = prefix + ".raw"
    lib.sampler_stop(raw.encode())
    print("post/write ms:", [(round(a, 1), round(b, 1)) for a, b in ts], flush=True)
    sampler.report(prefix, raw)
    os.unlink(out)


if __name__ == "__main__":
    main()
