"""Per-stage profile of one CLI run (`bwt.py ... --profile OUT.json`).

The stages are the reference's (bwt.py:3764-3789 load + index, 3892-3944
worker scan + post-processing, 4141-4198 save_results): each call the CLI
makes is timed here (wall ms, calls, bytes it moved) and the library adds its
own split of the same calls (`bwtmi_job_stage_ms`: scan, background index,
merge, refine..filter, render).  The library also opens a roctx range named
"bwtmi:<stage>" around every stage (csrc/trace.cpp), so a
`rocprofv3 --marker-trace --kernel-trace` run of the CLI attributes every
kernel and every host interval to one of these stages."""
from __future__ import annotations

import contextlib
import json
import os
import time
from typing import Dict, Optional

_active: Optional["Profile"] = None


class Profile:
    def __init__(self):
        self.t0 = time.perf_counter()
        self.stages: Dict[str, Dict[str, float]] = {}
        self.info: Dict[str, object] = {}

    @contextlib.contextmanager
    def stage(self, name: str, nbytes: int = 0):
        t = time.perf_counter()
        try:
            yield
        finally:
            s = self.stages.setdefault(name, {"ms": 0.0, "calls": 0, "bytes": 0})
            s["ms"] += (time.perf_counter() - t) * 1e3
            s["calls"] += 1
            s["bytes"] += int(nbytes)

    def add_bytes(self, name: str, nbytes: int) -> None:
        self.stages.setdefault(name, {"ms": 0.0, "calls": 0, "bytes": 0})["bytes"] += int(nbytes)

    def job_split(self, job) -> None:
        """The library's own split (bwtmi_job_stage_ms) of the last job calls."""
        ms = job.stage_ms()
        names = ["scan", "index", "nested", "dedup", "merge", "refine..filter", "render"]
        self.info["library_stage_ms"] = {n: round(v, 3) for n, v in zip(names, ms)}

    def write(self, path: str) -> None:
        out = dict(total_ms=round((time.perf_counter() - self.t0) * 1e3, 3),
                   stages={k: {"ms": round(v["ms"], 3), "calls": v["calls"], "bytes": v["bytes"]}
                           for k, v in self.stages.items()},
                   rank=int(os.environ.get("RANK", "0")), world=int(os.environ.get("WORLD_SIZE", "1")))
        out.update(self.info)
        with open(path, "w") as f:
            json.dump(out, f, indent=1)


def start() -> Profile:
    global _active
    _active = Profile()
    return _active


def active() -> Optional[Profile]:
    return _active


@contextlib.contextmanager
def stage(name: str, nbytes: int = 0):
    """Time a CLI stage when a profile is active (no-op otherwise)."""
    if _active is None:
        yield
        return
    with _active.stage(name, nbytes):
        yield
