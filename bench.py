#!/usr/bin/env python3
"""Benchmark of the hot path: Mbp/s indexed+scanned (Tier 1+2) on 100 Mbp
synthetic contigs, 1/2/4/8 GPUs (BASELINE.json `metric`).

Workload (with --progress so the reference's >50 Mbp Tier-2
gate does not turn the run into a header-only no-op): one 100,000,000 bp
synthetic contig per rank (seeded generator bwtmi/synth.py, contig k+1 on
rank k), default parameters (min_copies 3, max_unit_len 120 -> U = 1000).
Contigs are the sharding unit (one per GPU, weak scaling).

One step = one pass of the whole path over the resident contig(s):
  device FM index (SA, BWT, C, Occ, sampled SA, 8-mer hash)  [bwt.py:3053-3054]
  device strict adjacency scan + hit download                [bwt.py:3103-3106]
  native post-processing to the final records                [bwt.py:3928-3944]
  compound detection + STRfinder rows of the rank's own contig,
  written into one repeat.tab at offsets from an RCCL
  all-reduce of per-contig sizes (N > 1)                   [bwt.py:4141-4198]
  (sha256 and row count of the file are reported)
Inputs are resident in HBM before timing starts (uploaded during warmup).
"""
import argparse
import hashlib
import json
import os
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.abspath(__file__))
for _p in (REPO, os.path.join(REPO, "bwt-algorithm_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
PMC_SUMMARY = os.path.join(REPO, "profiles", "pmc_traffic.json")
# bench kernel-timer names -> kernel names in the rocprofv3 summaries
KERNEL_OF = {"radix_scatter_kv12": "k_scatter<u32>", "radix_scatter_kv16": "k_scatter<u64>",
             "radix_hist": "k_hist", "k_runs": "k_runs", "screen_levels": "k_level",
             "bwt_gather": "k_bwt", "occ_blocks": "k_occ_blocks", "sa_init_keys": "k_init_keys"}
CONTIG_BP = 100_000_000
FLANK = 30


def cpu_baseline(sample_bp: int):
    """Oracle port (C index + C strict scan + Python post-processing, 1 thread)
    on the first `sample_bp` bases of the rank-0 contig."""
    import oracle
    from oracle import post
    from bwtmi import synth
    seq = synth.generate_contig(sample_bp, 1, 0.0)
    t0 = time.perf_counter()
    trimmed = seq[FLANK:len(seq) - FLANK]
    oracle.Index(trimmed + b"$")
    U = max(120, min(len(trimmed) // 3, 1000))
    hits = oracle.strict_scan(trimmed, 1, U, 0, 3, threads=1)
    s = trimmed.decode()
    p = post.Pipeline({"contig1": s}, {"contig1": seq.decode()}, {"contig1": FLANK}, 3)
    recs = p.run(post.worker_records("contig1", s, hits))
    post.render(p, recs, "strfinder")
    dt = time.perf_counter() - t0
    return dict(value=round(sample_bp / 1e6 / dt, 5), unit="Mbp/s", cores=1, kind="port",
                sample=f"first {sample_bp:,} bp of contig1 (C3 workload): oracle index + strict scan "
                       f"+ post-processing + STRfinder render, 1 thread, {dt:.1f} s")


def fm_all_motifs(seq: bytes, reps: int = 5):
    """FM backward search over every canonical primitive ACGT motif of length
    1..10 (bwt.py:1369-1381 + 359-389; 145,338 patterns) on a device index of
    the rank's contig; outside the timed steps."""
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--contig-bp", type=int, default=CONTIG_BP)
    ap.add_argument("--cpu-sample-bp", type=int, default=1_000_000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-index", action="store_true", help="skip the FM index (scan-only step)")
    ap.add_argument("--no-fm", action="store_true", help="skip the all-motif FM search report")
    ap.add_argument("--stages", action="store_true", help="print per-stage times to stderr")
    ap.add_argument("--pmc-summary", default=PMC_SUMMARY,
                    help="tools/pmc_traffic.py output giving HBM bytes per launch (roofline.traffic)")
    a = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    td = None
    # BWTMI_BENCH_GLOO=1 (rehearsal aid on a box with fewer GPUs than ranks):
    # collectives over gloo on host tensors, rank r on device r mod #devices
    rehearsal = os.environ.get("BWTMI_BENCH_GLOO") == "1"
    if world > 1:
        import torch
        from bwtmi import dist
        td = dist.init("gloo" if rehearsal else None)   # RCCL (nccl backend) over xGMI

    from bwtmi import _lib, dist, synth
    from bwtmi.records import Job

    if rehearsal:
        local = local % max(1, _lib.device_count())
    ctx = _lib.ctx(local)
    # every rank registers every contig (fold-unit ids match across ranks) but
    # holds only its own sequence: rows are rendered and written by their owner
    job = Job(min_copies=3, max_unit_len=120, show_progress=True, tier2=True,
              build_index=not a.no_index, sa_sample=32)
    own_seq = b""
    for k in range(world):
        seq = synth.generate_contig(a.contig_bp, k + 1, 0.0) if k == rank else b""
        trim = FLANK if len(seq) > 2 * FLANK else 0
        job.add_contig(f"contig{k + 1}", seq, trim, trim)
        if k == rank:
            own_seq = seq
    job.select([rank])
    t_up = time.perf_counter()
    job.upload(ctx)                           # host -> HBM once; outside the timed region
    upload_ms = (time.perf_counter() - t_up) * 1000.0
    out_path = os.path.join(tempfile.gettempdir(), f"bwtmi_bench_{os.environ.get('MASTER_PORT', 'single')}.tab")
    dev = torch.device("cuda", local) if world > 1 and not rehearsal else None

    calls = {}

    def timed(name, fn, *args):
        t = time.perf_counter()
        r = fn(*args)
        calls[name] = calls.get(name, 0.0) + (time.perf_counter() - t) * 1e3
        return r

    def step():
        timed("reset", job.reset)
        job.select([rank])
        timed("scan", job.scan, ctx)
        timed("postprocess", job.postprocess)
        if world > 1:
            # each rank writes its own contig's rows at offsets from two
            # all-reduces of per-unit sizes (RCCL); no record leaves its GPU
            timed("write", dist.write_sharded, td, job, "strfinder", out_path, dev if dev is not None else "cpu")
        else:
            timed("write", job.write, "strfinder", out_path)     # repeat.tab, as the CLI writes it
        timed("index_wait", job.wait, ctx)    # the FM index build ran behind the host work
        return out_path

    def sync():
        if world > 1:
            torch.cuda.synchronize()
            td.barrier()
            torch.cuda.synchronize()

    for _ in range(a.warmup):
        step()
    calls.clear()
    _lib.kernel_stats(ctx, enable=True, reset=True)
    sync()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    sync()
    elapsed = time.perf_counter() - t0
    kstats = _lib.kernel_stats(ctx, enable=False, reset=True)
    stages = job.stage_ms()
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev if dev is not None else "cpu")
        td.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t.item())
    if a.stages:
        print(json.dumps(dict(rank=rank, stage_ms=stages, kernels=kstats)), file=sys.stderr)
    if rank != 0:
        if td is not None:
            td.barrier()
        return 0

    with open(out_path, "rb") as f:
        data = f.read()
    rows, digest = data.count(b"\n") - 1, hashlib.sha256(data).hexdigest()
    os.unlink(out_path)
    ms_step = elapsed / a.steps * 1000.0
    total_bp = world * a.contig_bp
    value = total_bp / 1e6 / (elapsed / a.steps)
    # dominant kernel = largest total device time in the timed steps
    dom = max(kstats.items(), key=lambda kv: kv[1][0]) if kstats else None
    roofline = None
    if dom:
        name, (kms, launches, kbytes) = dom
        achieved = kbytes / (kms / 1e3) / 1e9 if kms > 0 else 0.0
        traffic = None
        if a.pmc_summary and os.path.exists(a.pmc_summary) and a.contig_bp == CONTIG_BP:   # measured at C3
            with open(a.pmc_summary) as f:
                pk = json.load(f).get("kernels", {}).get(KERNEL_OF.get(name, name))
            if pk:
                traffic = pk["hbm_bytes_per_launch"]
        roofline = dict(bound="hbm", achieved=round(achieved, 2), peak=HBM_PEAK_GBS, unit="GB/s",
                        frac=round(achieved / HBM_PEAK_GBS, 5), traffic=traffic, kernel=name,
                        alg_bytes_per_launch=round(kbytes / launches), avg_launch_ms=round(kms / launches, 4),
                        launches_per_step=launches / a.steps)
    cpu = None if a.no_cpu_baseline else cpu_baseline(a.cpu_sample_bp)
    fm = None if a.no_fm else fm_all_motifs(own_seq)
    line = {
        "metric": "Mbp/s indexed+scanned (Tier1+2) on 100 Mbp synthetic FASTA, 1/2/4/8 GPU",
        "value": round(value, 3), "unit": "Mbp/s", "n_gpus": world, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": round(ms_step, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (seeded splitmix64 generator, bwtmi/synth.py)",
        "config": {"workload": "C3: one 100 Mbp synthetic contig per GPU, Tier1+2 defaults with "
                               "--progress (ungated), FM index + strict scan + post-processing + "
                               "STRfinder render", "contig_bp": a.contig_bp, "contigs": world,
                   "parallelism": f"contig-shard x{world}", "index": not a.no_index},
        "roofline": roofline,
        "cpu_baseline": cpu,
        "rows": rows,
        "output_sha256": digest,
        "stage_ms_last_step": {"scan+index": round(stages[0], 2), "index": round(stages[1], 2),
                               "nested": round(stages[2], 2), "dedup": round(stages[3], 2),
                               "merge": round(stages[4], 2), "refine..filter": round(stages[5], 2),
                               "render": round(stages[6], 2)},
        "kernels_ms_per_step": {k: round(v[0] / a.steps, 3) for k, v in sorted(kstats.items())},
        "h2d_upload_ms": round(upload_ms, 2),
        "fm_all_motifs_1_10": fm,
        "calls_ms_per_step": {k: round(v / a.steps, 2) for k, v in calls.items()},
        "value_incl_upload": round(total_bp / 1e6 / (elapsed / a.steps + upload_ms / 1e3), 3),
    }
    print(json.dumps(line))
    if td is not None:
        td.barrier()
    return 0


if __name__ == "__main__":
    sys.exit(main())
