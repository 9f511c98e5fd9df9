"""One rank's share of C4 at N=8 on this box: the 8 x
12.5 Mbp FASTA, LPT shard (world W, rank R) loaded by this process alone, the
bench step at N > 1 -- split load (pass 1 over the rank's 1/W of the file,
part tables all-gathered), index + scan, post-processing, and the SHARDED write
(bwtmi.dist.write_sharded: two all-reduces of per-unit counts, rank 0 sizes the
file, two barriers) -- with T host threads (T = cores/8 is the per-rank share
of a node whose host cores are split evenly among 8 GPU ranks).

The other ranks are stood in for by StandInComm: their contributions to the
four all-reduces (part-table sizes and words, per-unit rows and bytes) were
recorded in untimed steps of their own, and every collective of the timed step
still performs a collective of the same size -- an RCCL all-reduce at world 1
on this GPU (a launch and a stream wait) -- so its latency is inside the step.
Every rank of the world is timed (3 steps after a warm one) and the projection
uses the WORST step of the worst rank: a concurrent step costs the maximum over
ranks, which the worst single step bounds from above only if the ranks' steps
are independent (no data-path exchange); 100 Mbp / that step = projected 8-rank
C4 throughput.

Worlds other than 8 (C4_SHARD_WORLDS="8,4,2"): the same for the shards of a
2- or 4-rank run (4 or 2 contigs per rank).

usage: python tools/c4_shard.py OUT.json [threads ...]"""
import json, os, sys, tempfile, time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "bwt-algorithm_amd")]
FLANK = 30


class StandInComm:
    """The collectives of one rank's step (split load, sharded write) with the
    other W - 1 ranks' contributions recorded beforehand.  Calls are numbered
    within a step (begin_step): 0 / 1 the load's part-table all-gather (sizes,
    words), 2 / 3 the write's per-unit rows and bytes; barriers apart."""

    def __init__(self, fa, world, rank, rccl):
        import ctypes as C
        import numpy as np
        from bwtmi import _lib
        from bwtmi.records import Job
        self.world, self.rank, self.rccl = world, rank, rccl
        self.parts = []
        for r in range(world):
            j = Job()
            blob, nw = C.c_void_p(), C.c_int64()
            _lib.check(_lib.lib().bwtmi_job_fasta_scan_part(j.h, fa.encode(), world, r, C.byref(blob), C.byref(nw)))
            arr = np.ctypeslib.as_array(C.cast(blob, C.POINTER(C.c_int64)), shape=(nw.value,)).copy()
            _lib.lib().bwtmi_free(blob)
            self.parts.append(arr)
        self.others = {}   # call number -> sum of the other ranks' vectors
        self.own = {}      # call number -> this rank's vector (recorded)
        self.k = 0

    def begin_step(self):
        self.k = 0

    def _wire(self, a):
        import numpy as np
        if self.rccl is not None:   # a real collective of the same size: its latency is in the step
            self.rccl.allreduce(np.ascontiguousarray(a, dtype=np.int64))

    def allreduce(self, arr, op=0):
        import numpy as np
        a = np.ascontiguousarray(arr, dtype=np.int64)
        self._wire(a)
        k, self.k = self.k, self.k + 1
        if k == 0:   # part-table sizes in bytes
            return np.array([p.size * 8 for p in self.parts], dtype=np.int64)
        if k == 1:   # every rank's part table
            return np.concatenate(self.parts).astype(np.int64)
        self.own[k] = a.copy()
        return a + self.others.get(k, 0)

    def barrier(self):
        import numpy as np
        self._wire(np.zeros(1, dtype=np.int64))


def cgroup_cpu_us():
    """CPU time of this cgroup (all its threads) in microseconds, or None"""
    try:
        with open("/sys/fs/cgroup/cpu.stat") as f:
            for line in f:
                k, v = line.split()
                if k == "usage_usec":
                    return int(v)
    except (OSError, ValueError):
        pass
    return None


def main():
    out_json = sys.argv[1]
    tlist = [int(x) for x in sys.argv[2:]] or [2, 16]
    from bwtmi import _lib, comm as _comm, dist, synth
    from bwtmi.records import Job
    ctx = _lib.ctx(0)
    _lib.bind_host(ctx)
    rccl = _comm.RcclComm(_comm.Rendezvous(1, 0), 0) if os.environ.get("C4_SHARD_RCCL", "1") == "1" else None
    fa = os.path.join(tempfile.gettempdir(), "c4_shard.fa")
    synth.write_fasta(fa, [12_500_000] * 8, 0.0)
    out = os.path.join(tempfile.gettempdir(), "c4_shard.tab")
    worlds = [int(x) for x in os.environ.get("C4_SHARD_WORLDS", "8").split(",")]
    res = dict(workload="C4 shard: 8 x 12.5 Mbp FASTA, LPT shards of worlds %s" % worlds, host=_lib.host_info(),
               step="split load (part tables all-gathered) -> index + scan -> post-processing -> "
                    "dist.write_sharded (all-reduce of unit sizes, rank-0 truncate; each rank's pwrite behind the "
                    "next step as bench.py runs it, joined before the next sizes all-reduce, the last one joined "
                    "inside the last timed step; C4_SHARD_SYNC_WRITE=1: pwrite and barrier in the step)",
               collectives="RCCL all-reduce at world 1 per call" if rccl else "none (recorded results only)",
               runs=[])
    devload = os.environ.get("C4_SHARD_DEVLOAD", "1") == "1"   # device placement of the load (bench default)
    bg_write = os.environ.get("C4_SHARD_SYNC_WRITE", "0") != "1"
    res["device_load"] = devload
    for W, T in [(w, t) for w in worlds for t in tlist]:
        ranks = [int(x) for x in os.environ["C4_SHARD_RANKS"].split(",")] if os.environ.get("C4_SHARD_RANKS") else range(W)
        comms = {r: StandInComm(fa, W, r, rccl) for r in range(W)}
        jobs = {}
        for r in range(W):   # untimed: every rank's contributions to the write's all-reduces
            job = Job(min_copies=3, max_unit_len=120, show_progress=True, tier2=True,
                      build_index=os.environ.get("C4_SHARD_INDEX", "1") == "1",   # 0: what the index costs the host stages
                      sa_sample=32, threads=T)
            pc = comms[r]
            pc.begin_step()
            job.reset()
            job.load_fasta(fa, FLANK, W, r, pc, ctx if devload else None)
            job.upload(ctx)
            job.scan(ctx)
            job.postprocess()
            dist.write_sharded(pc, job, "strfinder", out)
            job.wait(ctx)
            jobs[r] = job
        for r in range(W):
            comms[r].others = {k: sum(comms[q].own[k] for q in range(W) if q != r) for k in comms[r].own}
        for r in ranks:             # every rank of the world: the worst one sets the projection
            job, pc = jobs[r], comms[r]
            calls = {}

            def timed(name, fn, *args):
                t = time.perf_counter()
                fn(*args)
                calls[name] = calls.get(name, 0.0) + (time.perf_counter() - t) * 1e3

            # the sharded write's pieces, timed apart (render / exchange / pwrite)
            def timed_method(nm, f):
                def g(*a, **kw):
                    t0 = time.perf_counter()
                    r = f(*a, **kw)
                    calls["w_" + nm] = calls.get("w_" + nm, 0.0) + (time.perf_counter() - t0) * 1e3
                    return r
                return g
            for meth in ("unit_rows", "render_units", "write_units"):
                if not hasattr(job, "_orig_" + meth):
                    setattr(job, "_orig_" + meth, getattr(job, meth))
                setattr(job, meth, timed_method(meth, getattr(job, "_orig_" + meth)))

            def step():
                pc.begin_step()
                timed("reset", job.reset)
                timed("load_fasta", job.load_fasta, fa, FLANK, W, r, pc, ctx if devload else None)
                timed("upload", job.upload, ctx)
                timed("scan", job.scan, ctx)
                timed("postprocess", job.postprocess)
                timed("write", dist.write_sharded, pc, job, "strfinder", out, bg_write)
                timed("index_wait", job.wait, ctx)
            step()
            calls.clear()
            ts = []
            cpu0 = cgroup_cpu_us()
            for q in range(3):
                t = time.perf_counter()
                step()
                if q == 2 and bg_write:   # the last step's file is whole inside its time
                    timed("write_join", dist.sharded_join, pc, job)
                ts.append((time.perf_counter() - t) * 1e3)
            cpu1 = cgroup_cpu_us()
            bp = sum(job.contig_weight(i) for i in job.select_shard(W, r))
            res["runs"].append(dict(world=W, threads=T, rank=r, shard_bp=bp, step_ms=round(max(ts), 2),
                                    median_ms=round(sorted(ts)[1], 2), mean_ms=round(sum(ts) / len(ts), 2),
                                    steps_ms=[round(x, 2) for x in ts], stage_ms=[round(x, 2) for x in job.stage_ms()],
                                    calls_ms={k: round(v / 3, 2) for k, v in calls.items()},
                                    cpu_ms_per_step=round((cpu1 - cpu0) / 3e3, 2) if cpu0 is not None and cpu1 is not None
                                    else None))
            print(json.dumps(res["runs"][-1]), flush=True)
    for W, T in [(w, t) for w in worlds for t in tlist]:
        worst = max(x["step_ms"] for x in res["runs"] if x["threads"] == T and x["world"] == W)
        res[f"worst_step_ms_{W}rank_at_{T}_threads"] = worst
        # what bench.py's line would see: the slowest rank's time over the steps
        res[f"worst_rank_mean_ms_{W}rank_at_{T}_threads"] = max(
            x["mean_ms"] for x in res["runs"] if x["threads"] == T and x["world"] == W)
        res[f"projected_{W}rank_mbp_per_s_at_{T}_threads_per_rank"] = round(100.0 / (worst / 1e3), 1)
    with open(out_json, "w") as f:
        json.dump(res, f, indent=1)
    os.unlink(fa)
    if os.path.exists(out):
        os.unlink(out)
    if rccl is not None:
        rccl.close()


if __name__ == "__main__":
    main()
