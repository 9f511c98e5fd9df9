#!/usr/bin/env python3
"""Benchmark of the hot path: Mbp/s indexed+scanned (Tier 1+2) on 100 Mbp
synthetic FASTA, 1/2/4/8 GPUs (BASELINE.json `metric`).

One step = the reference's CLI path from FASTA read to output file closed
(SURVEY.md §8(d)), per rank:
  native parallel FASTA parse of the rank's contigs      [bwt.py:3713-3756]
  H2D upload of the analysed sequences (pinned)
  device FM index (SA, BWT, C, Occ, sampled SA, 8-mer hash; runs behind
    the host stages)                                      [bwt.py:3053-3054]
  device strict adjacency scan + nested screening         [bwt.py:3103-3106]
  native post-processing to the final records             [bwt.py:3928-3944]
  compound detection + STRfinder rows written to repeat.tab
                                                          [bwt.py:4141-4198]
The synthetic FASTA is written to local disk once, before timing.

Workloads (`--workload`, default C3 on 1 GPU, C4 on N):
  C3  one 100,000,000 bp contig, defaults + --progress (the reference's
      >50 Mbp Tier-2 gate would otherwise make the output header-only);
      N > 1: one such FASTA per rank (weak scaling)
  C4  8 x 12,500,000 bp contigs in ONE FASTA; contigs sharded over the N
      ranks (longest-processing-time), each rank reads its contigs from the
      shared file and writes its rows into one shared repeat.tab at offsets
      from RCCL all-reduces of per-contig sizes (strong scaling)
  C5  C3 with 0.02 substitutions inside the planted arrays (the imperfect
      input; --no-mismatches is a no-op in the reference, bwt.py:3105)
The output sha256 is checked against the reference-pipeline golden
(tests/golden/expected_large.json) when the workload has one.
"""
import argparse
import hashlib
import json
import os
import platform
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.abspath(__file__))
for _p in (REPO, os.path.join(REPO, "bwt-algorithm_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
# VALU issue ceiling: 256 CUs x 4 SIMDs x 32 lanes/cycle x 2.4 GHz (MI355X_MICROARCH.md)
VALU_LANE_OPS_PEAK = 256 * 4 * 32 * 2.4e9
B_ALG_PER_BASE = 16.7          # compulsory HBM bytes per base, CLI path
PMC_SUMMARY = os.path.join(REPO, "profiles", "pmc_traffic.json")            # C3 / C5 kernels
PMC_SUMMARY_OF = {"C3N": os.path.join(REPO, "profiles", "pmc_traffic_C3N.json")}   # other workloads
# bench kernel-timer names -> kernel names in the rocprofv3 summaries
KERNEL_OF = {"radix_scatter_kv6": "k_scatter<u16,u32>", "radix_scatter_kv8": "k_scatter<u32,u32>", "radix_partition_kv8": "k_scatter<u32,u32>",
             "radix_scatter_kv12": "k_scatter<u64,u32>",
             "radix_scatter_kv16": "k_scatter<u64,u64>", "bwt_gather": "k_bwt", "occ_blocks": "k_occ_blocks",
             "sa_init_keys": "k_init_keys", "kmer_dna": "k_kmer_dna", "fm2_local": "k_fm2_local",
             "fm2_counts": "k_fm2_counts", "dna_ls_keys": "k_ls_wave",
             "radix_hist_k1": "k_hist_lb<u8>", "radix_hist_k2": "k_hist_lb<u16>", "radix_hist_k4": "k_hist_lb<u32>",
             "radix_hist_k8": "k_hist_lb<u64>", "k_scan": "k_scan_lb"}


def rocprof_name(timer: str) -> str:
    """bench kernel-timer name -> the kernel's short name in the rocprofv3 summaries"""
    if timer in KERNEL_OF:
        return KERNEL_OF[timer]
    return "k_" + timer if timer.startswith("dna_") else timer
FLANK = 30
# The reference itself (bwt.py --jobs 0 --progress, pure Python + numpy, no
# numba / pydivsufsort), timed in the build container -- it cannot run on the
# GPU box (tools/time_reference.py, profiles/r02/reference_cpu.json).  A
# one-contig file uses one core whatever the core count: Pool size
# min(cores, #contigs), bwt.py:3863-3864.
REFERENCE_CPU = dict(
    kind="reference", cores=1, host="build container, 8 vCPU Intel(R) Xeon(R) Processor, Python 3.10.12, numpy 2.2.6",
    cmd="bwt.py IN.fa -o OUT --jobs 0 --progress",
    runs=[dict(bp=10_000, seconds=35.8), dict(bp=1_000_000, seconds=5491.6)],
    value_1mbp=round(1.0 / 5491.6, 7), unit="Mbp/s",
    extrapolated_100mbp=dict(days=16.6, value=7.0e-5,
                             basis="5.5 us per strict-scan step x sum_L (n - 3L) + the O(k^2) nested loop"))
METRIC = "Mbp/s indexed+scanned (Tier1+2) on 100 Mbp synthetic FASTA, 1/2/4/8 GPU"
WORKLOADS = {
    "C3": dict(lengths=[100_000_000], sub_rate=0.0, shared=False, golden="C3p"),
    "C4": dict(lengths=[12_500_000] * 8, sub_rate=0.0, shared=True, golden="C4"),
    "C5": dict(lengths=[100_000_000], sub_rate=0.02, shared=False, golden="C5p"),
    # C3 with assembly gaps (bwtmi.synth GAP_PROFILES "n2": 3.8 % N in runs of
    # 10 bp - 958 kbp, ~1e4 single R/Y): the general-alphabet index and scan
    "C3N": dict(lengths=[100_000_000], sub_rate=0.0, shared=False, golden="C3Np", gaps="n2"),
}


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def cpu_baseline(sample_bp: int, sub_rate: float, threads: int, gaps=None):
    """Native CPU comparator on a bounded sample: the C oracle's index build
    (prefix doubling, each round's sort and re-rank on every thread) and OpenMP
    strict scan, then the product's multithreaded host
    post-processing + writer fed through bwtmi_job_add_hits."""
    import oracle
    from bwtmi import synth
    from bwtmi.records import Job
    seq = synth.generate_contig(sample_bp, 1, sub_rate, gaps=gaps)
    out = os.path.join(tempfile.gettempdir(), f"bwtmi_cpu_{os.getpid()}.tab")
    t0 = time.perf_counter()
    trimmed = seq[FLANK:len(seq) - FLANK]
    oracle.Index(trimmed + b"$", threads=threads)
    t1 = time.perf_counter()
    U = max(120, min(len(trimmed) // 3, 1000))
    hits = oracle.strict_scan(trimmed, 1, U, 0, 3, threads=threads)
    t2 = time.perf_counter()
    job = Job(min_copies=3, show_progress=True, threads=threads)
    job.add_contig("contig1", seq, FLANK, FLANK)
    job.add_hits(0, hits)
    job.postprocess()
    job.write("strfinder", out)
    t3 = time.perf_counter()
    os.unlink(out)
    dt = t3 - t0
    return dict(value=round(sample_bp / 1e6 / dt, 5), unit="Mbp/s", cores=threads, kind="port",
                sample=f"first {sample_bp:,} bp of contig1 (same generator): C oracle index + "
                       f"OpenMP strict scan + native post-processing and STRfinder write ({threads} threads), "
                       f"{dt:.1f} s",
                phases_s=dict(index=round(t1 - t0, 2), strict_scan=round(t2 - t1, 2),
                              post_and_write=round(t3 - t2, 2)),
                phase_threads=dict(index=threads, strict_scan=threads, post_and_write=threads),
                value_scan_and_post=round(sample_bp / 1e6 / (t3 - t1), 5),
                extrapolated_100mbp_s=round(dt * 100e6 / sample_bp, 1),
                reference_measured=REFERENCE_CPU)


def fm_all_motifs(seq: bytes, reps: int = 5):
    """FM backward search over every canonical primitive ACGT motif of length
    1..10 (bwt.py:1369-1381 + 359-389; 145,338 patterns) on a device index of
    the rank's first contig; outside the timed steps."""
    from bwtmi import BWTCore, MotifUtils
    core = BWTCore((seq[FLANK:len(seq) - FLANK] + b"$").decode("latin-1"))
    pats = [m for k in range(1, 11) for m in MotifUtils.enumerate_motifs(k)]
    blob, off = BWTCore.pack_patterns(pats)
    res = core.backward_search_packed(blob, off)
    t0 = time.perf_counter()
    for _ in range(reps):
        core.backward_search_packed(blob, off)
    dt = (time.perf_counter() - t0) / reps
    found = int((res[:, 0] >= 0).sum())
    core.clear()
    return dict(patterns=len(pats), found=found, ms=round(dt * 1e3, 3),
                mpatterns_per_s=round(len(pats) / dt / 1e6, 2))


def host_counters():
    """Process page faults / context switches and the cgroup's CPU-quota
    throttling (cpu.stat), read around the timed region: a host stage slowed by
    the quota or by page faulting shows here, not in the kernel times."""
    import resource
    ru = resource.getrusage(resource.RUSAGE_SELF)
    d = dict(minflt=ru.ru_minflt, majflt=ru.ru_majflt, nvcsw=ru.ru_nvcsw, nivcsw=ru.ru_nivcsw)
    try:
        with open("/sys/fs/cgroup/cpu.stat") as f:
            for line in f:
                k, v = line.split()
                if k in ("nr_throttled", "throttled_usec", "usage_usec"):
                    d["cg_" + k] = int(v)
    except (OSError, ValueError):
        pass
    return d


def cli_drop_in(fa: str, args, reps: int = 2):
    """The drop-in CLI (`bwt.py FA -o OUT ARGS`, bwt.py:4201-4370) run
    in-process on the workload's FASTA: wall time of each run (a fresh
    TandemRepeatFinder and job every time, so the first run carries the
    process's cold costs) and the output's sha256.  Outside the timed steps."""
    import contextlib
    import io
    from bwtmi import cli
    out = fa + ".cli.tab"
    times = []
    for _ in range(reps):
        t0 = time.perf_counter()
        with contextlib.redirect_stdout(io.StringIO()):
            rc = cli.main([fa, "-o", out] + list(args))
        times.append(round(time.perf_counter() - t0, 4))
        if rc != 0:
            raise RuntimeError(f"bwt.py CLI exited with {rc}")
    with open(out, "rb") as f:
        digest = hashlib.sha256(f.read()).hexdigest()
    os.unlink(out)
    return dict(argv=["bwt.py", "FA", "-o", "OUT"] + list(args), wall_s=times, output_sha256=digest)


def word_compares(n: int, U: int, mc: int = 3, lmin: int = 1):
    """32-position word compares of one contig's strict scan, split as
    strict_scan.hip launch_runs splits the unit lengths (bwt.py:1920):
      dense   k_runs, unit-length groups (32 L each) whose runs may hold no
              full aligned word: every word, sum_L ceil((n - L) / 32);
      sparse  k_runs_sparse, groups with K = (mc - 1) L >= 95: every s-th word
              with s = (K - 31) // 32 at the group's shortest L;
      dense_equivalent  every word for every L (what the sampling avoids).
    The sampled kernel's owner tests and streak-end scans (data-dependent)
    are not counted, so the rate from these counts is a lower bound."""
    lmax = min(U, n // mc)
    nw = (n + 31) // 32

    def stride(g):
        K = (mc - 1) * max(32 * g, lmin)
        return (K - 31) // 32 if K >= 95 else 0
    gs = max(1, lmin >> 5)
    while gs <= (lmax >> 5) and stride(gs) < 2:
        gs += 1
    lmax_dense = min(lmax, gs * 32 - 1)
    dense = sum((n - L + 31) // 32 for L in range(lmin, lmax_dense + 1))
    sparse = 0
    for g in range(gs, (lmax >> 5) + 1):
        lo, hi = max(32 * g, lmin), min(32 * g + 31, lmax)
        if hi >= lo:
            sparse += (hi - lo + 1) * ((nw + stride(g) - 1) // stride(g))
    every = sum((n - L + 31) // 32 for L in range(lmin, lmax + 1))
    return dict(dense=dense, sparse=sparse, dense_equivalent=every)


def launch_ranks(n: int, argv, script: str = None) -> int:
    """`bench.py --gpus N` without an external launcher: N rank processes of
    this script, one per GPU (bwtmi.dist.launch_ranks: RANK / LOCAL_RANK /
    WORLD_SIZE / MASTER_* in their environment, a failing rank stops its
    peers).  This parent never touches the GPU.  Rank 0 prints the line."""
    from bwtmi import dist
    return dist.launch_ranks(n, [sys.executable, script or os.path.abspath(__file__)] + list(argv))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", choices=["auto"] + sorted(WORKLOADS), default="auto")
    ap.add_argument("--contig-bp", type=int, default=0, help="override every contig length (tests)")
    ap.add_argument("--cpu-sample-bp", type=int, default=30_000_000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-index", action="store_true", help="skip the FM index (scan-only step)")
    ap.add_argument("--no-fm", action="store_true", help="skip the all-motif FM search report")
    ap.add_argument("--no-cli", action="store_true", help="skip the in-process drop-in CLI timing")
    ap.add_argument("--stages", action="store_true", help="print per-stage times to stderr")
    ap.add_argument("--host-load", action="store_true",
                    help="whole-file load on the host + upload (default: built on the device from the file image)")
    ap.add_argument("--time-all-kernels", action="store_true",
                    help="time every launch in the timed steps (default: only the dominant kernel; the table from the warmup)")
    ap.add_argument("--sync-write", action="store_true",
                    help="write each step's file before the step ends (bwtmi_job_write) instead of behind the next step")
    ap.add_argument("--pmc-summary", default=None,
                    help="tools/pmc_traffic.py output giving HBM bytes per launch (roofline.traffic)")
    a = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        return launch_ranks(a.gpus, sys.argv[1:])
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if a.gpus > 1 and world != a.gpus:
        print(f"bench.py: --gpus {a.gpus} but the launcher started WORLD_SIZE={world} ranks", file=sys.stderr)
        return 2
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    wl_name = a.workload if a.workload != "auto" else ("C3" if world == 1 else "C4")
    wl = dict(WORKLOADS[wl_name])
    if a.contig_bp:
        wl["lengths"] = [a.contig_bp] * len(wl["lengths"])
    shared = wl["shared"]

    from bwtmi import _lib, comm as _comm, dist, synth
    from bwtmi.records import Job

    # BWTMI_BENCH_GLOO=1 (rehearsal with more ranks than GPUs): collectives over
    # the host transport, rank r on device r mod #devices
    rehearsal = os.environ.get("BWTMI_BENCH_GLOO") == "1"
    c = _comm.get("host" if rehearsal else None) if world > 1 else None
    if rehearsal:
        local = local % max(1, _lib.device_count())
    ctx = _lib.ctx(local)
    _lib.bind_host(ctx)        # host threads next to the GPU (the library never does it by itself)
    host = _lib.host_info()

    # input FASTA on local disk, written once before timing
    tmp = tempfile.gettempdir()
    tag = os.environ.get("MASTER_PORT", "single")
    if shared:
        fa = os.path.join(tmp, f"bwtmi_bench_{wl_name}_{tag}.fa")
        if rank == 0:
            synth.write_fasta(fa, wl["lengths"], wl["sub_rate"], gaps=wl.get("gaps"))
        out = os.path.join(tmp, f"bwtmi_bench_{wl_name}_{tag}.tab")
    else:   # one contig (index rank + 1) per rank, own FASTA, own output
        fa = os.path.join(tmp, f"bwtmi_bench_{wl_name}_{tag}_r{rank}.fa")
        synth.write_fasta(fa, wl["lengths"], wl["sub_rate"], first_index=rank + 1, gaps=wl.get("gaps"))
        out = os.path.join(tmp, f"bwtmi_bench_{wl_name}_{tag}_r{rank}.tab")
    if c is not None:
        c.barrier()
    load_world, load_rank = (world, rank) if shared else (1, 0)

    job = Job(min_copies=3, max_unit_len=120, show_progress=True, tier2=True,
              build_index=not a.no_index, sa_sample=32)
    calls = {}

    def timed(name, fn, *args):
        t = time.perf_counter()
        r = fn(*args)
        calls[name] = calls.get(name, 0.0) + (time.perf_counter() - t) * 1e3
        return r

    def step():
        timed("reset", job.reset)
        # shared FASTA over N ranks: each scans 1/N of it, the part tables are all-gathered
        # one whole file: the sequences are built on the device from the file image
        # and the host copy is written behind the scan (bwtmi_job_load_fasta_dev)
        timed("load_fasta", job.load_fasta, fa, FLANK, load_world, load_rank, c if load_world > 1 else None,
              None if a.host_load else ctx)
        timed("upload", job.upload, ctx)
        timed("scan", job.scan, ctx)
        timed("postprocess", job.postprocess)
        if shared and world > 1:
            # each rank writes its own contigs' rows at offsets from two
            # all-reduces of per-unit sizes; no record leaves its GPU
            # (the pwrite lands behind the next step: joined before the next
            # write's sizes all-reduce, and by sync() inside the timed region)
            timed("write", dist.write_sharded, c, job, "strfinder", out, not a.sync_write)
        else:
            # repeat.tab, as the CLI writes it; the call returns once the rows are
            # formatted and the job's writer finishes the file behind the next
            # step's load and scan (bwtmi_job_write_async).  The next step joins it
            # before rewriting the file ("write_join"), and sync() joins the last
            # one inside the timed region, so every step's file is whole in it.
            timed("write_join", job.write_join)
            timed("write", job.write, "strfinder", out, not a.sync_write)
        timed("index_wait", job.wait, ctx)    # the FM index build ran behind the host work

    def sync():
        job.write_join()   # this rank's file write (every rank's, after the barrier below)
        _lib.lib().bwtmi_device_sync(local)
        if c is not None:
            c.barrier()

    # Every launch is timed during the warmup steps after the first (the
    # kernels_ms_per_step table and the choice of the dominant kernel); in the
    # timed steps only the dominant kernel is (its live roofline): an event pair
    # per launch leaves ~10 us of device idle between dependent launches, 0.7 ms
    # in the scan call's 73 launches (r06ae, tools/scan_gaps.py).
    warm_stats, warm_steps = {}, 0
    for w in range(a.warmup):
        if w == min(1, a.warmup - 1):
            _lib.kernel_stats(ctx, enable=True, reset=True)
        step()
        warm_steps += w >= min(1, a.warmup - 1)
    if a.warmup:
        warm_stats = _lib.kernel_stats(ctx, enable=False, reset=True)
    dominant = ""
    if warm_stats and not a.time_all_kernels:
        with_b = {k: v for k, v in warm_stats.items() if v[2] > 0}
        dominant = max(warm_stats.items(), key=lambda kv: kv[1][0])[0]
        if warm_stats[dominant][2] <= 0 and with_b:
            dominant = max(with_b.items(), key=lambda kv: kv[1][0])[0]
    _lib.kernel_stats_filter(ctx, dominant)
    calls.clear()
    _lib.kernel_stats(ctx, enable=True, reset=True)
    sync()
    host0 = host_counters()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    sync()
    elapsed = time.perf_counter() - t0
    host1 = host_counters()
    kstats = _lib.kernel_stats(ctx, enable=False, reset=True)
    _lib.kernel_stats_filter(ctx, "")
    # the per-kernel table: the warmup's when the timed steps timed only the dominant kernel
    table, table_steps = (warm_stats, warm_steps) if dominant else (kstats, a.steps)
    stages = job.stage_ms()
    if c is not None:
        import numpy as np
        elapsed = float(c.allreduce(np.array([elapsed], dtype=np.float64), _comm.MAX)[0])
    if a.stages:
        print(json.dumps(dict(rank=rank, stage_ms=stages, kernels=kstats, calls=calls)), file=sys.stderr)

    def cleanup():
        for p in ((out, fa) if (not shared or rank == 0) else ()):
            try:
                os.unlink(p)
            except OSError:
                pass

    if rank != 0:
        if c is not None:
            c.barrier()      # rank 0 has read the shared output
        cleanup()
        return 0

    with open(out, "rb") as f:
        data = f.read()
    rows, digest = data.count(b"\n") - 1, hashlib.sha256(data).hexdigest()
    golden = None
    gpath = os.path.join(REPO, "tests", "golden", "expected_large.json")
    if not a.contig_bp and os.path.exists(gpath):
        with open(gpath) as f:
            g = json.load(f).get(wl["golden"])
        if g and (shared or world == 1):
            golden = dict(name=wl["golden"], sha256=g["out_sha256"], rows=g["out_rows"],
                          match=g["out_sha256"] == digest)
    total_bp = sum(wl["lengths"]) * (1 if shared else world)
    ms_step = elapsed / a.steps * 1000.0
    value = total_bp / 1e6 / (elapsed / a.steps)
    per_call = {k: v / a.steps for k, v in calls.items()}

    # dominant kernel = largest total device time (over the warmup's timed
    # launches; or the timed steps' with --time-all-kernels), its live time
    # from the timed steps
    dev_ms = sum(v[0] for v in table.values()) / max(1, table_steps) * a.steps
    roofline = None
    with_bytes = {k: v for k, v in kstats.items() if v[2] > 0}
    if with_bytes:
        name, (kms, launches, kbytes) = max(kstats.items(), key=lambda kv: kv[1][0])
        if kbytes <= 0:   # the largest kernel has no byte model: fall back to the largest modelled one
            name, (kms, launches, kbytes) = max(with_bytes.items(), key=lambda kv: kv[1][0])
        achieved = kbytes / (kms / 1e3) / 1e9 if kms > 0 else 0.0
        traffic = None
        pmc = a.pmc_summary or PMC_SUMMARY_OF.get(wl_name, PMC_SUMMARY)
        if os.path.exists(pmc) and wl_name in ("C3", "C5", "C3N") and not a.contig_bp:
            with open(pmc) as f:
                pk = json.load(f).get("kernels", {}).get(rocprof_name(name))
            if pk:
                traffic = pk["hbm_bytes_per_launch"]
        roofline = dict(bound="hbm", achieved=round(achieved, 2), peak=HBM_PEAK_GBS, unit="GB/s",
                        frac=round(achieved / HBM_PEAK_GBS, 5), traffic=traffic, kernel=name,
                        alg_bytes_per_launch=round(kbytes / launches), avg_launch_ms=round(kms / launches, 4),
                        launches_per_step=launches / a.steps,
                        share_of_device_time=round(kms / dev_ms, 4) if dev_ms else None)
        # the write pattern's own ceiling, measured apart (tools/scatter_ceiling.hip): context for
        # frac, which stays against the 8 TB/s HBM peak
        ceil = os.path.join(REPO, "profiles", "r05", "scatter_ceiling_r05x.json")
        if name in ("radix_scatter_kv8", "radix_partition_kv8") and os.path.exists(ceil):
            with open(ceil) as f:
                cj = json.load(f)
            roofline["pattern_ceiling"] = dict(
                unit="GB/s", copy=round(cj["copy_tbs"] * 1e3), runs32_xcd=round(cj["runs_skew_xcd_tbs"] * 1e3),
                source="profiles/r05/scatter_ceiling_r05x.json: 1.6 GB per launch as a streaming copy, and as "
                       "256 misaligned runs of 32 pairs per 8192-pair tile in the product's XCD tile order")
    # strict scan: the word compares k_runs (dense groups) and k_runs_sparse
    # (sampled groups) perform, over the time of both plus k_streak_end, against
    # the VALU issue ceiling; the all-words count only as a labelled reference
    mine = job.select_shard(load_world, load_rank) if shared else range(job.contig_count())
    wc = dict(dense=0, sparse=0, dense_equivalent=0)
    for i in mine:
        w = job.contig_weight(i)
        for k, v in word_compares(w, max(120, min(w // 3, 1000))).items():
            wc[k] += v
    scan_names = ("k_runs", "k_runs_sparse", "k_streak_end")
    scan_ms = sum(table[k][0] for k in scan_names if k in table) / max(1, table_steps)
    scan_rate = None
    if scan_ms > 0:
        done = wc["dense"] + wc["sparse"]
        per_s = done / (scan_ms / 1e3)
        scan_rate = dict(word_compares_per_step=done, dense_compares=wc["dense"], sampled_compares=wc["sparse"],
                         kernels=list(scan_names),
                         kernels_ms_per_step=round(scan_ms, 3), gcompares_per_s=round(per_s / 1e9, 2),
                         valu_lane_ops_peak=VALU_LANE_OPS_PEAK,
                         frac_of_valu_issue_at_1_op_per_compare=round(per_s / VALU_LANE_OPS_PEAK, 5),
                         note="owner tests and streak-end scans of the sampled groups (data-dependent) are not "
                              "counted: a lower bound",
                         dense_equivalent=dict(word_compares=wc["dense_equivalent"],
                                               gcompares_per_s=round(wc["dense_equivalent"] / (scan_ms / 1e3) / 1e9, 2),
                                               meaning="every word for every unit length: the work the sampling "
                                                       "avoids, not work done"))
    e2e_gbs = B_ALG_PER_BASE * total_bp / (elapsed / a.steps) / 1e9
    cpu = None if a.no_cpu_baseline else cpu_baseline(a.cpu_sample_bp, wl["sub_rate"], host["threads_per_rank"],
                                                        wl.get("gaps"))
    fm = None
    if not a.no_fm:
        first = min(i for i in range(job.contig_count()) if job.contig_info(i)[1] > 0)
        fm = fm_all_motifs(job.contig_seq(first))
    cli = None
    if world == 1 and not shared and not a.no_cli:
        cli = cli_drop_in(fa, ["--progress", "--jobs", "0"])
        cli["vs_step"] = round(min(cli["wall_s"]) * 1e3 / ms_step, 2)
        cli["golden_match"] = golden["sha256"] == cli["output_sha256"] if golden else None
    load_up = per_call.get("load_fasta", 0.0) + per_call.get("upload", 0.0)
    line = {
        "metric": METRIC,
        "value": round(value, 3), "unit": "Mbp/s", "n_gpus": world, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": round(ms_step, 3), "higher_is_better": True,
        "scaling": "strong" if shared else "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic FASTA on local disk (seeded splitmix64 generator, bwtmi/synth.py), "
                "read and parsed inside every step",
        "config": {"workload": f"{wl_name}: " + {
                       "C3": "one 100 Mbp synthetic contig per GPU, Tier1+2 defaults with --progress (ungated)",
                       "C4": "8 x 12.5 Mbp contigs in one FASTA, contigs sharded over the GPUs",
                       "C5": "one 100 Mbp contig with 0.02 substitutions in the planted arrays, --progress",
                       "C3N": "one 100 Mbp contig with assembly gaps (3.8 % N in runs up to 958 kbp, "
                              "single R/Y), --progress"}[wl_name]
                   + "; FASTA read -> FM index + strict scan + post-processing -> STRfinder repeat.tab closed",
                   "contig_bp": wl["lengths"][0], "contigs": len(wl["lengths"]) * (1 if shared else world),
                   "parallelism": f"contig-shard x{world}", "index": not a.no_index,
                   "load": "host" if a.host_load else "device",
                   "write": ("in the step" if a.sync_write else
                             "sharded: each rank's pwrite behind the next step, joined before the next write's "
                             "sizes all-reduce and before the timed region ends" if shared and world > 1 else
                             "finished behind the next step's load and scan, joined before the file "
                             "is rewritten and before the timed region ends")},
        "roofline": roofline,
        "e2e_roofline": {"b_alg_bytes_per_base": B_ALG_PER_BASE, "achieved_gbs": round(e2e_gbs, 2),
                         "peak_gbs": HBM_PEAK_GBS * world, "frac": round(e2e_gbs / (HBM_PEAK_GBS * world), 6)},
        "strict_scan_rate": scan_rate,
        "cpu_baseline": cpu,
        "host": dict(host, nproc=os.cpu_count(), cpu_model=cpu_model()),
        "rows": rows,
        "output_sha256": digest,
        "golden": golden,
        "stage_ms_last_step": {"scan": round(stages[0], 2), "index": round(stages[1], 2),
                               "nested": round(stages[2], 2), "dedup": round(stages[3], 2),
                               "merge": round(stages[4], 2), "refine..filter": round(stages[5], 2),
                               "render": round(stages[6], 2)},
        "device_ms_per_step": round(dev_ms / a.steps, 3),
        "kernels_ms_per_step": {k: round(v[0] / max(1, table_steps), 3) for k, v in
                                sorted(table.items(), key=lambda kv: -kv[1][0])},
        "kernels_ms_source": (f"warmup steps 2-{a.warmup} (every launch timed); in the timed steps only "
                              f"{dominant} is timed" if dominant else "timed steps (every launch timed)"),
        "calls_ms_per_step": {k: round(v, 2) for k, v in per_call.items()},
        "host_per_step": {k: round((host1[k] - host0[k]) / a.steps, 1) for k in host1 if k in host0},
        "value_resident_text": round(total_bp / 1e6 / ((ms_step - load_up) / 1e3), 3) if ms_step > load_up else None,
        "fm_all_motifs_1_10": fm,
        "cli_drop_in": cli,
    }
    print(json.dumps(line))
    if c is not None:
        c.barrier()
    cleanup()
    return 0


if __name__ == "__main__":
    sys.exit(main())
