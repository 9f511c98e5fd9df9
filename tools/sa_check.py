#!/usr/bin/env python3
"""Suffix array of the shared-prefix run texts (bwtmi.synth.shared_prefix_runs)
on the device against the oracle, outside pytest, so that another library build
(BWTMI_LIB=...) can be checked with the same inputs: an A/B of a suffix-sort
fix.  Prints one JSON line per text; exit status 1 when any differs."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "bwt-algorithm_amd")]

import numpy as np  # noqa: E402

import oracle  # noqa: E402
from bwtmi import BWTCore, synth  # noqa: E402


def texts():
    for alpha in (b"ACGT", b"ACGTNRY"):
        yield f"{alpha.decode()}_s1", synth.shared_prefix_runs(alpha, 1)
        yield f"{alpha.decode()}_short_x3", synth.shared_prefix_runs(
            alpha, 2, run_lengths=(16, 17, 20, 31, 32, 33), prefix_lengths=(32, 64)) * 3
        big = b"".join(synth.shared_prefix_runs(alpha, s, run_lengths=(16, 24, 31, 40, 63), prefix_lengths=(32, 64))
                       for s in range(3, 40))
        yield f"{alpha.decode()}_1M", big[:1_000_000]


def main() -> int:
    bad = 0
    for name, t in texts():
        text = t + b"$"
        sa = BWTCore(text.decode("latin-1")).suffix_array
        ref = oracle.Index(text).sa
        diff = np.nonzero(sa != ref)[0]
        print(json.dumps(dict(text=name, n=len(text), rows_differing=int(len(diff)),
                              first=int(diff[0]) if len(diff) else None)), flush=True)
        bad += len(diff) > 0
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
