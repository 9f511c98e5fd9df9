"""`bwt.py` command line (bwt.py:4201-4370): same positional argument, the
same 16 options and defaults, the same output files."""
from __future__ import annotations

import argparse
import os
import sys
from typing import Optional

from .finder import TandemRepeatFinder


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(
        description="Advanced BWT-based Tandem Repeat Finder with Imperfect Repeat Support "
                    "(MI355X-native engine)",
        formatter_class=argparse.RawDescriptionHelpFormatter)
    p.add_argument("reference", help="Reference genome FASTA file")
    p.add_argument("-o", "--output", default="repeat.tab", help="Output file (default: repeat.tab)")
    p.add_argument("--format", choices=["bed", "vcf", "trf_table", "trf_dat", "strfinder"],
                   default="strfinder", help="Output format (default: strfinder)")
    p.add_argument("--tier1", action="store_true", help="Enable tier 1 only (short repeats, 1-9bp)")
    p.add_argument("--tier3", action="store_true", help="Enable tier 3 (very long repeats, kb+)")
    p.add_argument("--long-reads", help="Long reads file for tier 3")
    p.add_argument("--sa-sample", type=int, default=32, help="Suffix array sampling rate (default: 32)")
    p.add_argument("--progress", action="store_true", help="Show progress bars where applicable")
    p.add_argument("--jobs", type=int, default=4,
                   help="Parallel workers (default: 4, 0=all, -1=sequential); results are identical")
    p.add_argument("--no-mismatches", action="store_true",
                   help="Disable mismatch tolerance (exact matches only)")
    p.add_argument("--max-motif-len", type=int, default=9, help="Maximum motif length for tier 1 (default: 9)")
    p.add_argument("--min-period", type=int, default=10, help="Minimum period for tier 2 (default: 10)")
    p.add_argument("--max-period", type=int, default=1000, help="Maximum period for tier 2 (default: 1000)")
    p.add_argument("--max-unit-len", type=int, default=120,
                   help="Maximum unit length for tier 2 long repeat detection (default: 120)")
    p.add_argument("--min-copies", type=int, default=3, help="Minimum number of copies required (default: 3)")
    p.add_argument("--min-entropy", type=float, default=1.0,
                   help="Minimum Shannon entropy to avoid low-complexity (default: 1.0)")
    p.add_argument("--profile", metavar="JSON", default=None,
                   help="write per-stage wall ms / calls / bytes of this run to JSON (rank r of N: JSON.rankR)")
    p.add_argument("--flank-trim", type=int, default=30,
                   help="Trim N bp from each end before analysis (default: 30, use 0 to disable)")
    return p


def _read_long_reads(path: str):
    reads, cur = [], ""
    with open(path) as f:
        for line in f:
            line = line.strip()
            if line.startswith(">") or line.startswith("@"):
                if cur:
                    reads.append(cur)
                    cur = ""
            elif not line.startswith("+"):
                cur += line.upper()
    if cur:
        reads.append(cur)
    return reads


# inputs below this size stay in one process: a rank's start-up (interpreter,
# HIP and RCCL initialisation, ~1-2 s) outweighs what more GPUs save on them
LAUNCH_MIN_BYTES = 32 << 20


def _self_launch(a, argv) -> Optional[int]:
    """The reference fans contigs out to a Pool of `--jobs` workers (0 = all
    CPUs, -1 = sequential; bwt.py:3850-3912, 3863-3864, 4336-4358).  Here a
    worker is a GPU: without an external launcher, `--jobs N|0` starts
    min(N or #GPUs, #GPUs, #contigs) rank processes of this CLI, one per GPU,
    that shard the contigs' fold units and write the shared output file
    (find_and_write_sharded).  Returns their exit code, or None to run in
    this process: one rank's worth of work, `--jobs -1`, Tier 3 (its records
    join the scan of every contig in one process), a small input, or
    BWTMI_CLI_LAUNCH=0.  This process touches no GPU before the launch (the
    devices are counted in a child; the records by the library's host-only
    bwtmi_fasta_count_records -- loading the library and that call leave no
    /dev/kfd or DRM descriptor open, checked on the box).  BWTMI_CLI_RANKS=N forces N ranks over
    the host transport, rank r on device r mod #GPUs (a rehearsal of an
    N-GPU node on fewer GPUs)."""
    from . import dist
    if dist.is_distributed() or a.jobs == -1 or a.tier3 or os.environ.get("BWTMI_CLI_LAUNCH", "1") == "0":
        return None
    forced = int(os.environ.get("BWTMI_CLI_RANKS", "0") or 0)
    if not forced:
        try:
            if os.path.getsize(a.reference) < LAUNCH_MIN_BYTES:
                return None
        except OSError:
            return None
    cap = forced or (a.jobs if a.jobs > 0 else 1 << 20)
    n = min(cap, dist.count_fasta_records(a.reference, limit=cap + 1))
    if n <= 1:
        return None
    ndev = dist.count_devices_in_child()
    if ndev < 1:
        return None
    if not forced:
        n = min(n, ndev)
        if n <= 1:
            return None
    script = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bwt.py")

    def env(r):
        e = {"BWTMI_CLI_CHILD": "1"}
        if forced:
            e.update(BWTMI_COMM="host", BWTMI_DEVICE=str(r % ndev))
        return e
    return dist.launch_ranks(n, [sys.executable, script] + list(argv), env)


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    a = build_parser().parse_args(argv)
    child = os.environ.get("BWTMI_CLI_CHILD") == "1"
    tier2 = not a.tier1                                   # bwt.py:4257-4262
    tiers = "Tier 1 (short repeats)" if a.tier1 else "Tier 1 + Tier 2 (short + medium repeats)"
    if a.tier3:
        tiers += " + Tier 3 (very long repeats)"
    if not child:
        print("BWT-based Tandem Repeat Finder")
        print("=" * 60)
        print(f"Reference:    {a.reference}")
        print(f"Output:       {a.output} ({a.format} format)")
        print(f"Tiers:        {tiers}")
        print(f"Engine:       libbwtmi on MI355X (gfx950)")
        print()
        sys.stdout.flush()
        rc = _self_launch(a, argv)
        if rc is not None:
            return rc
    # the process that does the work binds its host threads next to its GPU
    # (bwtmi_open reads the switch; a library user's affinity is never touched)
    from . import _lib
    _lib.knob("NUMA_BIND", 1)
    from . import profile
    prof = profile.start() if a.profile else None
    rc = _run(a, tier2)
    if prof is not None:
        path = a.profile if int(os.environ.get("WORLD_SIZE", "1")) == 1 else f"{a.profile}.rank{os.environ.get('RANK', '0')}"
        prof.write(path)
    return rc


def _run(a, tier2) -> int:
    finder = TandemRepeatFinder(a.reference, a.sa_sample, show_progress=a.progress,
                                allow_mismatches=not a.no_mismatches, max_motif_length=a.max_motif_len,
                                min_period=a.min_period, max_period=a.max_period,
                                min_copies=a.min_copies, min_entropy=a.min_entropy,
                                flank_trim=a.flank_trim, max_unit_len=a.max_unit_len)
    from . import dist
    if dist.is_distributed() and not a.tier3:
        # one process per GPU: each rank loads and analyses its own fold units
        # and writes their rows into the shared output (no torch, no record gather)
        n = finder.find_and_write_sharded(tier2, a.output, a.format)
        if dist.init().rank == 0:
            print()
            print("=" * 60)
            print(f"Completed! Found {n} total tandem repeats.")
            print(f"Results saved to {a.output}")
        return 0
    sequences = finder.load_reference()
    if os.environ.get("BWTMI_SKIP_INDEX", "0") != "1":
        finder.build_indices(sequences)
    long_reads = _read_long_reads(a.long_reads) if (a.long_reads and a.tier3) else []
    if a.jobs != -1:
        repeats = finder.find_tandem_repeats_parallel(True, tier2, a.tier3, long_reads or None, None)
    else:
        repeats = finder.find_tandem_repeats(True, tier2, a.tier3, long_reads or None)
    if dist.is_distributed() and dist.init().rank != 0:
        return 0
    finder.save_results(repeats, a.output, a.format)
    print()
    print("=" * 60)
    print(f"Completed! Found {len(repeats)} total tandem repeats.")
    print(f"Results saved to {a.output}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
