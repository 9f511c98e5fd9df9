"""Multi-GPU sharding over contigs: one process per GPU, no PyTorch.

The reference parallelises over contigs with multiprocessing.Pool
(bwt.py:3894-3912) and every post-processing step is per chromosome
(SURVEY.md §8(e)).  Here each rank owns whole *fold units* (contigs with
equal natural sort keys, bwt.py:22-36 -- normally one contig each), assigned
by longest-processing-time greedy over their analysed lengths
(bwtmi_job_select_shard; `assign` below is the same rule in Python, for
tests).  A rank loads only its own contigs' bases from the shared FASTA,
runs the device scan and the native post-processing for them, and writes its
rows into the shared output file at byte offsets that two all-reduces of
per-unit counts give every rank (write_sharded) -- records never move between
GPUs.  The collectives go through bwtmi.comm (RCCL over xGMI on MI355X, a
host transport for CPU tests).

The module API (find_tandem_repeats* returning records) gathers the final
records to rank 0 instead (run_sharded), through the same collective.
"""
from __future__ import annotations

import os
from typing import Callable, List, Optional, Sequence

import numpy as np

from . import _lib, comm as _comm


def is_distributed() -> bool:
    """True under a multi-rank launch (WORLD_SIZE > 1)."""
    return int(os.environ.get("WORLD_SIZE", "1")) > 1


def init(transport: Optional[str] = None):
    """The process's communicator (bwtmi.comm.get)."""
    return _comm.get(transport)


def natural_units(names: Sequence[str]) -> List[List[int]]:
    """Group contig ids whose natural sort keys collide (bwt.py:22-36)."""
    import re

    def key(v):
        out = []
        for part in re.split(r"(\d+)", str(v)):
            if part:
                out.append((0, int(part)) if part.isdigit() else (1, part.lower()))
        return tuple(out)

    groups = {}
    for i, n in enumerate(names):
        groups.setdefault(key(n), []).append(i)
    return [groups[k] for k in sorted(groups)]


def assign(units: List[List[int]], weights: Sequence[int], world: int) -> List[List[int]]:
    """Longest-processing-time greedy over units; deterministic."""
    w = [sum(weights[c] for c in u) for u in units]
    order = sorted(range(len(units)), key=lambda k: (-w[k], k))
    load = [0] * world
    out: List[List[int]] = [[] for _ in range(world)]
    for k in order:
        r = min(range(world), key=lambda x: (load[x], x))
        load[r] += w[k]
        out[r].extend(units[k])
    return [sorted(x) for x in out]


def write_sharded(comm, job, fmt: str, path: str) -> int:
    """Write the output file from every rank's own fold units, without moving
    records between ranks.  The file is the units' rows in unit (natural-key)
    order (bwt.py:4147-4150) and each unit lives on exactly one rank, so two
    all-reduces of per-unit counts (rows for VCF ids, then bytes) give every
    rank its byte offsets; rank 0 sizes the file and writes the header.
    Returns the file size."""
    rows = comm.allreduce(job.unit_rows())
    row_base = np.concatenate([[0], np.cumsum(rows)[:-1]]).astype(np.int64)
    local = job.render_units(fmt, row_base)
    sizes = comm.allreduce(np.ascontiguousarray(local[1:]))
    header = int(local[0])
    offsets = np.concatenate([[0, header], header + np.cumsum(sizes)[:-1]]).astype(np.int64)
    total = header + int(sizes.sum())
    if comm.rank == 0:
        # sized in place: every byte of [0, total) is written below, so an
        # existing file is overwritten (reusing its page-cache pages) and cut
        with open(path, "r+b" if os.path.isfile(path) else "wb") as f:
            f.truncate(total)
    comm.barrier()
    job.write_units(path, offsets, write_header=(comm.rank == 0))
    comm.barrier()
    return total


def run_sharded(finder, job, scan_fn: Optional[Callable] = None):
    """Shard `job`'s contigs over the ranks; returns rank 0's RepeatList (other
    ranks get an empty one).  `scan_fn(job, ids)` overrides the device scan
    (CPU tests feed checker hits through it)."""
    c = init()
    shard = job.select_shard(c.world, c.rank)
    if scan_fn is not None:
        scan_fn(job, shard)
    else:
        job.scan(_lib.ctx(int(os.environ.get("LOCAL_RANK", "0"))))
    from .finder import TandemRepeatFinder
    TandemRepeatFinder._report_errors(job)   # the worker's ERROR line per failed contig (bwt.py:3137-3141)
    job.postprocess()
    if scan_fn is None:
        job.wait(_lib.ctx(int(os.environ.get("LOCAL_RANK", "0"))))
    blobs = _comm.allgather_bytes(c, job.export())
    job.reset()
    job.select(None)
    if c.rank == 0:
        for b in blobs:
            job.import_records(b)
    return job.records()
