"""TandemRepeatFinder -- the reference's orchestrator (bwt.py:3144-4198) with
the same constructor, methods and results, running on one MI355X device per
process.

  load_reference      native FASTA loader (bwt.py:3713-3756)
  build_indices       device FM index per contig (bwt.py:3758-3790)
  find_tandem_repeats / find_tandem_repeats_parallel
                      device strict scan per contig + native post-processing
                      (bwt.py:3792-3954); under a multi-rank launch
                      the contigs are sharded over ranks (bwtmi.dist)
  save_results        native writers incl. compound detection (bwt.py:4141-4198)
"""
from __future__ import annotations

import os
import sys
import time
from collections.abc import MutableMapping
from typing import Dict, List, Optional

from . import _lib
from .core import BWTCore
from .records import Job, RepeatList, TandemRepeat


class _ContigMap(MutableMapping):
    """`sequences` / `full_sequences` of a loaded finder: name -> str, decoded
    from the native loader's bytes on first access only (the CLI path never
    reads them, so no per-base Python work is done at 100 Mbp).  Same keys,
    order and duplicate-name rule as load_reference (bwt.py:3713-3756)."""

    def __init__(self, job: Job, trimmed: bool):
        self._job, self._trimmed = job, trimmed
        self._ids: Dict[str, int] = {}
        for i in range(job.contig_count()):
            self._ids[job.contig_info(i)[0]] = i          # a later duplicate wins, in place
        self._vals: Dict[str, str] = {}
        self._over = set()    # names assigned by the caller (their value replaces the loader's bytes)

    def raw(self, name: str) -> bytes:
        if name in self._over:
            return self._vals[name].encode("latin-1")
        name_, fl, tl, tr = self._job.contig_info(self._ids[name])
        full = self._job.contig_seq(self._ids[name])
        return full[tl:fl - tr] if self._trimmed else full

    def contig_id(self, name: str) -> int:
        return self._ids[name]

    def __getitem__(self, name: str) -> str:
        v = self._vals.get(name)
        if v is None:
            if name not in self._ids:
                raise KeyError(name)
            v = self._vals[name] = self.raw(name).decode("latin-1")
        return v

    def __setitem__(self, name: str, value: str) -> None:
        if name not in self._ids:
            self._ids[name] = -1
        self._vals[name] = value
        self._over.add(name)

    def __delitem__(self, name: str) -> None:
        del self._ids[name]
        self._vals.pop(name, None)
        self._over.discard(name)

    def __iter__(self):
        return iter(self._ids)

    def __len__(self):
        return len(self._ids)


class _DeferredCore(BWTCore):
    """BWTCore over a loaded contig + '$', built on the device on first use.
    build_indices of the reference (bwt.py:3758-3790) builds a parent index per
    contig that the default path never reads (only Tier 3 does);
    the worker's own index (bwt.py:3053-3054) is built by the job behind the
    post-processing.  So the parent's indices are deferred, not dropped: any
    attribute or query builds it exactly as BWTCore(seq + '$') would."""

    def __init__(self, seqs: "_ContigMap", name: str, sa_sample_rate: int, device: Optional[int]):
        object.__setattr__(self, "_deferred", (seqs, name, sa_sample_rate, device))

    def _build(self) -> None:
        seqs, name, rate, dev = object.__getattribute__(self, "_deferred")
        object.__setattr__(self, "_deferred", None)
        BWTCore.__init__(self, seqs.raw(name) + b"$", rate, device=dev)

    def __getattr__(self, attr):
        if attr.startswith("__") or object.__getattribute__(self, "_deferred") is None:
            raise AttributeError(attr)
        self._build()
        return getattr(self, attr)

    def __del__(self):
        if object.__getattribute__(self, "_deferred") is None:
            BWTCore.__del__(self)


class TandemRepeatFinder:
    def __init__(self, reference_file: str, sa_sample_rate: int = 32, show_progress: bool = False,
                 allow_mismatches: bool = True, max_motif_length: int = 9, min_period: int = 10,
                 max_period: int = 1000, min_copies: int = 3, min_entropy: float = 1.0,
                 flank_trim: int = 30, max_unit_len: int = 120, device: Optional[int] = None,
                 threads: int = 0):
        self.reference_file = reference_file
        self.sa_sample_rate = sa_sample_rate
        self.bwt_cores: Dict[str, BWTCore] = {}
        self.sequences: Dict[str, str] = {}
        self.show_progress = show_progress
        self.allow_mismatches = allow_mismatches      # no effect on results (bwt.py:3105)
        self.max_motif_length = max_motif_length
        self.min_period = min_period
        self.max_period = max_period
        self.min_copies = min_copies
        self.min_entropy = min_entropy
        self.flank_trim = max(0, flank_trim)
        self.max_unit_len = max_unit_len
        self.trim_offsets: Dict[str, int] = {}
        self.full_sequences: Dict[str, str] = {}
        self.device = device
        self.threads = threads
        self.job: Optional[Job] = None

    # ------------------------------------------------------------------ input
    def _new_job(self, tier2: bool = True) -> Job:
        # the worker's FM index (bwt.py:3053-3054) is built by the job on the
        # device, behind the host post-processing (BWTMI_SKIP_INDEX=1: not at all)
        build = os.environ.get("BWTMI_SKIP_INDEX", "0") != "1"
        return Job(min_copies=self.min_copies, max_unit_len=self.max_unit_len,
                   show_progress=self.show_progress, tier2=tier2, threads=self.threads,
                   build_index=build, sa_sample=self.sa_sample_rate)

    def load_reference(self) -> Dict[str, str]:
        job = self._new_job()
        # with a device the analysed sequences are built there from the file
        # image and the host copies are written behind the scan
        # (bwtmi_job_load_fasta_dev); BWTMI_HOST_LOAD=1 loads on the host only
        dev = None
        if os.environ.get("BWTMI_HOST_LOAD", "0") != "1":
            try:
                dev = _lib.ctx(self.device) if _lib.device_count() > 0 else None
            except _lib.BwtmiError:
                dev = None
        job.load_fasta(self.reference_file, self.flank_trim, dev_ctx=dev)
        self.job = job
        self.full_sequences = _ContigMap(job, trimmed=False)
        self.sequences = _ContigMap(job, trimmed=True)
        self.trim_offsets = {}
        for i in range(job.contig_count()):
            name, fl, tl, tr = job.contig_info(i)
            self.trim_offsets[name] = tl
        return self.sequences

    def build_indices(self, sequences: Dict[str, str]):
        """One device FM index per contig over seq + '$' (bwt.py:3758-3790).
        Sequences of this finder's own load_reference get deferred indices
        (_DeferredCore); any other mapping is indexed now."""
        print("Building BWT indices...")
        t0 = time.time()
        items = list(sequences.keys())
        own = isinstance(sequences, _ContigMap) and sequences is self.sequences
        for i, chrom in enumerate(items, 1):
            pct = (i - 1) / len(items) * 100
            if own:
                self.bwt_cores[chrom] = _DeferredCore(sequences, chrom, self.sa_sample_rate, self.device)
                print(f"\r  {pct:5.1f}% Index for {chrom} queued", end="", flush=True)
            else:
                seq = sequences[chrom]
                print(f"\r  {pct:5.1f}% Building index for {chrom} ({len(seq):,} bp)", end="", flush=True)
                self.bwt_cores[chrom] = BWTCore(seq + "$", self.sa_sample_rate, device=self.device)
        print(f"\r  100.0% BWT indices built for {len(items)} chromosome(s) - {time.time() - t0:.1f}s     ")
        print()

    # ------------------------------------------------------------------ search
    def _run(self, enable_tier2: bool, enable_tier3: bool, long_reads, parallel: bool = True) -> RepeatList:
        if self.job is None:
            self.load_reference()
        job = self.job
        job.reset()
        if parallel and enable_tier3 and long_reads:
            self._tier3(job, long_reads)
        if self.min_copies == 0 and enable_tier2:
            # the reference worker raises ZeroDivisionError and returns [] (bwt.py:3095, 3137-3141)
            for name in job.names:
                print(f"ERROR processing chromosome {name}: integer division or modulo by zero")
        job.set_tier2(enable_tier2)
        from . import dist
        if dist.is_distributed():
            return dist.run_sharded(self, job)
        job.scan(_lib.ctx(self.device))
        self._report_errors(job)
        job.postprocess()
        job.wait(_lib.ctx(self.device))     # the worker's FM index build ran behind post-processing
        return job.records()

    @staticmethod
    def _report_errors(job) -> None:
        """The worker's failure convention (bwt.py:3137-3141): a contig whose
        device work failed is reported and contributes no records."""
        for cid, msg in job.contig_errors().items():
            print(f"ERROR processing chromosome {job.names[cid]}: {msg}")
            print(f"bwtmi: contig {job.names[cid]!r} failed on the device: {msg}", file=sys.stderr)

    def _tier3(self, job, long_reads) -> None:
        """Tier 3 (bwt.py:3917-3924, parallel mode only): every built index
        anchors the long reads; the records join that contig's strict hits
        ahead of nested suppression (bwtmi_index_tier3 as_input=1)."""
        from .tiers import Tier3LongReadFinder
        print("\nTier 3 processing (serial)...")
        ids = {name: i for i, name in enumerate(job.names)}   # load_reference: the last duplicate wins
        for chrom, core in self.bwt_cores.items():
            if chrom not in ids:
                raise KeyError(f"Tier 3: index {chrom!r} has no loaded sequence")
            Tier3LongReadFinder(core, show_progress=self.show_progress)._run(long_reads, job, ids[chrom], True)

    def find_and_write_sharded(self, enable_tier2: bool, output_file: str, format_type: str) -> int:
        """Multi-GPU CLI path: every rank scans and post-processes its own fold
        units and writes them into `output_file` at offsets from an exchange of
        per-unit sizes (bwtmi.dist.write_sharded) -- records never leave their
        rank.  Returns the total number of records (all ranks)."""
        import numpy as np
        from . import dist
        c = dist.init()
        if self.job is None:
            job = self._new_job()
            job.load_fasta(self.reference_file, self.flank_trim, c.world, c.rank, comm=c)
            self.job = job
        job = self.job
        job.reset()
        job.set_tier2(enable_tier2)
        job.select_shard(c.world, c.rank)
        job.scan(_lib.ctx(self.device))
        self._report_errors(job)
        job.postprocess()
        total = int(c.allreduce(np.array([job.count()], dtype=np.int64))[0])
        dist.write_sharded(c, job, format_type, output_file)
        job.wait(_lib.ctx(self.device))
        return total

    def find_tandem_repeats(self, enable_tier1: bool = True, enable_tier2: bool = True,
                            enable_tier3: bool = False, long_reads: Optional[List[str]] = None) -> RepeatList:
        res = self._run(enable_tier2, enable_tier3, long_reads, parallel=False)   # no Tier 3 (bwt.py:3792-3848)
        print(f"Analysis complete! Found {len(res)} total repeats.")
        return res

    def find_tandem_repeats_parallel(self, enable_tier1: bool = True, enable_tier2: bool = True,
                                     enable_tier3: bool = False, long_reads: Optional[List[str]] = None,
                                     n_jobs: Optional[int] = None) -> RepeatList:
        res = self._run(enable_tier2, enable_tier3, long_reads)
        print(f"Analysis complete! Found {len(res)} unique repeats.")
        return res

    # ------------------------------------------------------------------ output
    def save_results(self, repeats, output_file: str, format_type: str = "bed"):
        if format_type not in _lib.FMT:
            raise ValueError(f"unknown format {format_type}")
        if isinstance(repeats, RepeatList):
            repeats.job.write(format_type, output_file)
            return
        # any other list of records (e.g. a filtered RepeatList): rendered by a
        # job holding the same contigs, without touching this finder's records
        job = self._new_job()
        if repeats:
            if not self.full_sequences:
                self.load_reference()
            for name, full in self.full_sequences.items():
                t = self.trim_offsets.get(name, 0)
                job.add_contig(name, full.encode("latin-1"), t, t)
            job.set_records(list(repeats), self.full_sequences)
        job.write(format_type, output_file)
