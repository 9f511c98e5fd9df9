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
import signal
import socket
import subprocess
import sys
import time
from typing import Callable, Dict, List, Optional, Sequence

import numpy as np

from . import _lib, comm as _comm


def is_distributed() -> bool:
    """True under a multi-rank launch (WORLD_SIZE > 1)."""
    return int(os.environ.get("WORLD_SIZE", "1")) > 1


def launch_ranks(n: int, cmd: Sequence[str], extra_env: Optional[Callable[[int], Dict[str, str]]] = None) -> int:
    """Start `cmd` as n rank processes of one job on this node (RANK /
    LOCAL_RANK / WORLD_SIZE / LOCAL_WORLD_SIZE / MASTER_* in their environment,
    rank r on GPU r) and wait for them; returns the first failing exit code,
    else 0.  A failing rank stops its peers (they would wait for it in a
    collective forever).  The caller must not have touched the GPU: the ranks
    are fresh processes, as the reference's Pool workers are
    (bwt.py:3850-3912)."""
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), BWTMI_RDZV_PORT=str(port))
        if extra_env is not None:
            env.update(extra_env(r))
        procs.append(subprocess.Popen(list(cmd), env=env, start_new_session=True))
    rc = 0
    # a SIGTERM / SIGHUP to this launcher (kill, a scheduler's soft stop) reaches
    # the ranks too: they run in sessions of their own and would outlive it
    forwarded = {}

    def forward(signum, frame):
        for q in procs:
            if q.poll() is None:
                try:
                    os.killpg(q.pid, signum)
                except ProcessLookupError:
                    pass
        raise SystemExit(128 + signum)
    for sig in (signal.SIGTERM, signal.SIGHUP):
        try:
            forwarded[sig] = signal.signal(sig, forward)
        except ValueError:   # not the main thread: no handlers
            pass
    try:
        live = list(procs)
        while live:
            time.sleep(0.02)
            for p in list(live):
                code = p.poll()
                if code is None:
                    continue
                live.remove(p)
                if code != 0 and rc == 0:
                    rc = code if code > 0 else 128 - code
                    print(f"bwtmi: rank {procs.index(p)} exited with {code}; stopping the other ranks",
                          file=sys.stderr)
                    for q in live:
                        try:
                            os.killpg(q.pid, signal.SIGTERM)
                        except ProcessLookupError:
                            pass
    finally:
        for sig, old in forwarded.items():
            signal.signal(sig, old)
        for p in procs:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, signal.SIGKILL)
                except ProcessLookupError:
                    pass
                p.wait()
    return rc


def count_devices_in_child() -> int:
    """GPUs this process could use, counted in a child process so that the
    caller never initialises HIP (it may still start rank processes); 0 when
    there is none or the library cannot be loaded."""
    pkg = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = ("import sys; sys.path.insert(0, %r)\n"
            "try:\n    from bwtmi import _lib; print(_lib.device_count())\n"
            "except Exception:\n    print(0)\n") % pkg
    try:
        out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
        return int(out.stdout.strip().splitlines()[-1])
    except (subprocess.SubprocessError, ValueError, IndexError, OSError):
        return 0


def count_fasta_records(path: str, limit: int = 1 << 20) -> int:
    """Header lines ('>' at a line start) of a FASTA file, counted up to
    `limit` -- an upper bound on its fold units (bwt.py:3713-3756; natural-key
    collisions and duplicate names only merge units).  The native parallel
    count (bwtmi_fasta_count_records, host only); 0 for an unreadable file."""
    from ._lib import lib
    n = int(lib().bwtmi_fasta_count_records(os.fsencode(path), int(limit)))
    return max(n, 0)


def _count_fasta_records_py(path: str, limit: int = 1 << 20) -> int:
    """The same count in Python (two mmap scans) -- the tests' cross-check."""
    import mmap
    try:
        with open(path, "rb") as f:
            if os.fstat(f.fileno()).st_size == 0:
                return 0
            with mmap.mmap(f.fileno(), 0, access=mmap.ACCESS_READ) as m:
                n = 1 if m[:1] == b">" else 0
                for sep in (b"\n>", b"\r>"):
                    pos = m.find(sep)
                    while pos >= 0 and n < limit:
                        n += 1
                        pos = m.find(sep, pos + 2)
                return n
    except OSError:
        return 0


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


def write_sharded(comm, job, fmt: str, path: str, background: bool = False) -> int:
    """Write the output file from every rank's own fold units, without moving
    records between ranks.  The file is the units' rows in unit (natural-key)
    order (bwt.py:4147-4150) and each unit lives on exactly one rank, so an
    all-reduce of per-unit byte counts gives every rank its byte offsets (VCF
    also needs the rows before each unit for its TR ids: one all-reduce of
    per-unit row counts first); rank 0 writes the header and sizes the file.
    Sizing commutes with the writes -- every rank writes inside [0, total), and
    ftruncate to total neither moves nor drops those bytes whenever it lands --
    so only the end of the write needs a barrier.  Returns the file size.

    background=True: each rank's pwrite runs behind the caller, and there is
    no barrier: every rank joins its previous write before it enters the sizes
    all-reduce, so once that returns no rank's earlier write is still landing
    when rank 0 sizes the file and the ranks write again.  The caller joins
    the last one with sharded_join()."""
    row_base = None
    if fmt == "vcf":
        rows = comm.allreduce(job.unit_rows())
        row_base = np.concatenate([[0], np.cumsum(rows)[:-1]]).astype(np.int64)
    local = job.render_units(fmt, row_base)
    if background:
        job.write_join()   # this rank's previous write (the all-reduce below then orders every rank's)
    sizes = comm.allreduce(np.ascontiguousarray(local[1:]))
    header = int(local[0])
    offsets = np.concatenate([[0, header], header + np.cumsum(sizes)[:-1]]).astype(np.int64)
    total = header + int(sizes.sum())
    if comm.rank == 0:
        # sized in place: every byte of [0, total) is written, so an existing file
        # is overwritten (reusing its page-cache pages) and cut
        fd = os.open(path, os.O_WRONLY | os.O_CREAT, 0o644)
        try:
            os.ftruncate(fd, total)
        finally:
            os.close(fd)
    job.write_units(path, offsets, write_header=(comm.rank == 0), background=background)
    if not background:
        comm.barrier()
    return total


def sharded_join(comm, job) -> None:
    """Wait for this rank's background write (write_sharded(background=True)),
    then for every rank's: afterwards the file is whole on every rank."""
    job.write_join()
    comm.barrier()


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
