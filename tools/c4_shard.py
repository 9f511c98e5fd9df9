"""One rank's share of C4 at N=8 on this box: the 8 x 12.5 Mbp
FASTA, LPT shard (world 8, rank R) loaded by this process alone, the bench
step (load -> index + scan -> post-processing -> write of the shard's rows)
with T host threads -- T = cores/8 is the per-rank share of a node whose host
cores are split evenly among 8 GPU ranks.  Projected 8-rank C4 throughput =
100 Mbp / the slowest shard's step (ranks share no data path; the only
collectives are two small all-reduces in the sharded write).

Worlds other than 8 (C4_SHARD_WORLDS="8,4,2"): the same for the shards of a
2- or 4-rank run (4 or 2 contigs per rank).

usage: python tools/c4_shard.py OUT.json [threads ...]"""
import json, os, sys, tempfile, time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "bwt-algorithm_amd")]
FLANK = 30


class PartsComm:
    """Stands in for the other 7 ranks of the split load: their part tables are
    computed once, before timing (on a real node they come from the ranks
    themselves, through two small all-reduces); allreduce returns what the
    collective would."""

    def __init__(self, fa, world, rank):
        import ctypes as C
        import numpy as np
        from bwtmi import _lib
        from bwtmi.records import Job
        self.world, self.rank = world, rank
        self.parts = []
        for r in range(world):
            j = Job()
            blob, nw = C.c_void_p(), C.c_int64()
            _lib.check(_lib.lib().bwtmi_job_fasta_scan_part(j.h, fa.encode(), world, r, C.byref(blob), C.byref(nw)))
            arr = np.ctypeslib.as_array(C.cast(blob, C.POINTER(C.c_int64)), shape=(nw.value,)).copy()
            _lib.lib().bwtmi_free(blob)
            self.parts.append(arr)

    def allreduce(self, arr, op=0):
        import numpy as np
        if arr.size == self.world:   # sizes
            return np.array([p.size * 8 for p in self.parts], dtype=np.int64)
        return np.concatenate(self.parts).astype(np.int64)


def main():
    out_json = sys.argv[1]
    tlist = [int(x) for x in sys.argv[2:]] or [2, 16]
    from bwtmi import _lib, synth
    from bwtmi.records import Job
    ctx = _lib.ctx(0)
    _lib.bind_host(ctx)
    fa = os.path.join(tempfile.gettempdir(), "c4_shard.fa")
    synth.write_fasta(fa, [12_500_000] * 8, 0.0)
    out = os.path.join(tempfile.gettempdir(), "c4_shard.tab")
    worlds = [int(x) for x in os.environ.get("C4_SHARD_WORLDS", "8").split(",")]
    res = dict(workload="C4 shard: 8 x 12.5 Mbp FASTA, LPT shards of worlds %s" % worlds, host=_lib.host_info(),
               runs=[])
    split = os.environ.get("C4_SHARD_SPLIT", "1") == "1"   # the split loader (bench / CLI at N > 1)
    res["split_load"] = split
    devload = os.environ.get("C4_SHARD_DEVLOAD", "1") == "1"   # device placement of the load (bench default)
    res["device_load"] = devload
    for W, T in [(w, t) for w in worlds for t in tlist]:
        ranks = [int(x) for x in os.environ["C4_SHARD_RANKS"].split(",")] if os.environ.get("C4_SHARD_RANKS") else range(W)
        for r in ranks:             # every rank of the world: the worst one sets the projection
            job = Job(min_copies=3, max_unit_len=120, show_progress=True, tier2=True,
                      build_index=os.environ.get("C4_SHARD_INDEX", "1") == "1",   # 0: what the index costs the host stages
                      sa_sample=32, threads=T)

            calls = {}

            def timed(name, fn, *args):
                t = time.perf_counter()
                fn(*args)
                calls[name] = calls.get(name, 0.0) + (time.perf_counter() - t) * 1e3

            pc = PartsComm(fa, W, r) if split else None

            def step():
                timed("reset", job.reset)
                timed("load_fasta", job.load_fasta, fa, FLANK, W, r, pc, ctx if devload else None)
                timed("upload", job.upload, ctx)
                timed("scan", job.scan, ctx)
                timed("postprocess", job.postprocess)
                timed("write", job.write, "strfinder", out)
                timed("index_wait", job.wait, ctx)
            step()
            calls.clear()
            ts = []
            for _ in range(3):
                t = time.perf_counter()
                step()
                ts.append((time.perf_counter() - t) * 1e3)
            bp = sum(job.contig_weight(i) for i in job.select_shard(W, r))
            ms = sorted(ts)[1]
            res["runs"].append(dict(world=W, threads=T, rank=r, shard_bp=bp, step_ms=round(ms, 2),
                                    steps_ms=[round(x, 2) for x in ts], stage_ms=[round(x, 2) for x in job.stage_ms()],
                                    calls_ms={k: round(v / 3, 2) for k, v in calls.items()}))
            print(json.dumps(res["runs"][-1]), flush=True)
    for W, T in [(w, t) for w in worlds for t in tlist]:
        worst = max(x["step_ms"] for x in res["runs"] if x["threads"] == T and x["world"] == W)
        res[f"projected_{W}rank_mbp_per_s_at_{T}_threads_per_rank"] = round(100.0 / (worst / 1e3), 1)
    with open(out_json, "w") as f:
        json.dump(res, f, indent=1)
    os.unlink(fa)
    if os.path.exists(out):
        os.unlink(out)


if __name__ == "__main__":
    main()
