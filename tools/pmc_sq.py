"""Per-kernel SQ counters from one rocprofv3 --pmc pass (stall analysis).

usage: python tools/pmc_sq.py DIR [kernel-substring ...]

Sums each counter over the dispatches of each kernel (short names as in
pmc_traffic.py) and prints them with the fractions of SQ_WAVE_CYCLES
(MI355X_MICROARCH.md: WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY ~ WAVE_CYCLES)."""
import csv
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_traffic import short  # noqa: E402


def main(argv):
    d = argv[1]
    pats = argv[2:]
    files = glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True)
    acc = {}
    for f in files:
        with open(f, newline="") as fh:
            for row in csv.DictReader(fh):
                k = short(row.get("Kernel_Name", ""))
                if pats and not any(p in k for p in pats):
                    continue
                c = row["Counter_Name"]
                acc.setdefault(k, {}).setdefault(c, 0.0)
                acc[k][c] += float(row["Counter_Value"])
    for k, cs in sorted(acc.items()):
        wc = cs.get("SQ_WAVE_CYCLES", 0.0)
        parts = []
        for c, v in sorted(cs.items()):
            fr = f" ({v / wc:.2f})" if wc and c.startswith(("SQ_WAIT", "SQ_ACTIVE", "SQ_LDS")) else ""
            parts.append(f"{c}={v:.4g}{fr}")
        print(k, " ".join(parts))


if __name__ == "__main__":
    main(sys.argv)
