"""Multi-GPU sharding over contigs: one process per GPU (torch.distributed,
RCCL over xGMI on MI355X, gloo for CPU tests).

The reference parallelises over contigs with multiprocessing.Pool
(bwt.py:3894-3912) and every post-processing step is per chromosome
(SURVEY.md §8(e)).  Here each rank owns whole *fold units* (contigs with
equal natural sort keys -- normally one contig), runs the device scan and the
native post-processing for them, and ships its final records to rank 0 in
one all-gather of byte buffers -- the only collective on the path.  Rank 0
imports them and renders; output is identical to a single-GPU run.
"""
from __future__ import annotations

import os
from typing import Callable, List, Optional, Sequence

from . import _lib


def _torch_dist():
    import torch.distributed as td
    return td


def is_distributed() -> bool:
    """True under a multi-rank launch.  Never imports torch itself: the
    single-GPU path stays torch-free (a cold torch import costs minutes)."""
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        return True
    import sys
    td = sys.modules.get("torch.distributed")
    return bool(td is not None and td.is_available() and td.is_initialized() and td.get_world_size() > 1)


def init(backend: Optional[str] = None):
    import torch
    td = _torch_dist()
    if not td.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
        td.init_process_group(backend=backend, init_method="env://")
    return td


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


def gather_bytes(td, blob: bytes, device) -> List[bytes]:
    """All-gather variable-size byte buffers (sizes first, then padded payload)."""
    import torch
    world = td.get_world_size()
    n = torch.tensor([len(blob)], dtype=torch.int64, device=device)
    sizes = [torch.zeros(1, dtype=torch.int64, device=device) for _ in range(world)]
    td.all_gather(sizes, n)
    sizes = [int(s.item()) for s in sizes]
    m = max(sizes) if sizes else 0
    buf = torch.zeros(max(m, 1), dtype=torch.uint8, device=device)
    if blob:
        buf[:len(blob)] = torch.frombuffer(bytearray(blob), dtype=torch.uint8).to(device)
    parts = [torch.zeros(max(m, 1), dtype=torch.uint8, device=device) for _ in range(world)]
    td.all_gather(parts, buf)
    return [bytes(p[:s].cpu().numpy().tobytes()) for p, s in zip(parts, sizes)]


def _allreduce_sum(td, arr, device):
    import numpy as np
    import torch
    t = torch.from_numpy(np.ascontiguousarray(arr, dtype=np.int64)).to(device)
    td.all_reduce(t, op=td.ReduceOp.SUM)
    return t.cpu().numpy()


def write_sharded(td, job, fmt: str, path: str, device="cpu") -> int:
    """Write the output file from every rank's own fold units, without moving
    records between ranks.  The file is the units' rows in unit (natural-key)
    order (bwt.py:4147-4150) and each unit lives on exactly one rank, so two
    all-reduces of per-unit counts (rows for VCF ids, then bytes) give every
    rank its byte offsets; rank 0 sizes the file and writes the header.
    Returns the file size."""
    import numpy as np
    rank = td.get_rank()
    rows = _allreduce_sum(td, job.unit_rows(), device)
    row_base = np.concatenate([[0], np.cumsum(rows)[:-1]]).astype(np.int64)
    local = job.render_units(fmt, row_base)
    sizes = _allreduce_sum(td, local[1:], device)
    header = int(local[0])
    offsets = np.concatenate([[0, header], header + np.cumsum(sizes)[:-1]]).astype(np.int64)
    total = header + int(sizes.sum())
    if rank == 0:
        # sized in place: every byte of [0, total) is written below, so an
        # existing file is overwritten (reusing its page-cache pages) and cut
        with open(path, "r+b" if os.path.isfile(path) else "wb") as f:
            f.truncate(total)
    td.barrier()
    job.write_units(path, offsets, write_header=(rank == 0))
    td.barrier()
    return total


def run_sharded(finder, job, scan_fn: Optional[Callable] = None):
    """Shard `job`'s contigs over the ranks; returns rank 0's RepeatList (other
    ranks get an empty one).  `scan_fn(job, ids)` overrides the device scan
    (CPU tests feed checker hits through it)."""
    import torch
    td = init()
    rank, world = td.get_rank(), td.get_world_size()
    infos = [job.contig_info(i) for i in range(job.contig_count())]
    weights = [fl - tl - tr for (_, fl, tl, tr) in infos]
    shard = assign(natural_units([x[0] for x in infos]), weights, world)[rank]
    job.select(shard)
    if scan_fn is not None:
        scan_fn(job, shard)
    else:
        job.scan(_lib.ctx(int(os.environ.get("LOCAL_RANK", "0"))))
    job.postprocess()
    if scan_fn is None:
        job.wait(_lib.ctx(int(os.environ.get("LOCAL_RANK", "0"))))
    blob = job.export()
    device = torch.device("cuda", torch.cuda.current_device()) if td.get_backend() == "nccl" else "cpu"
    blobs = gather_bytes(td, blob, device)
    job.reset()
    job.select(None)
    if rank == 0:
        for b in blobs:
            job.import_records(b)
    return job.records()
