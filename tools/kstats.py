"""Summarise a rocprofv3 kernel_stats.csv: per kernel calls, total ms, average us
(names shortened to the kernel identifier and its template arguments).
usage: python tools/kstats.py FILE.csv [top]"""
import csv
import re
import sys


def short(name):
    m = re.match(r"(?:void )?(?:bwtmi::)?(?:\(anonymous namespace\)::)?([A-Za-z_0-9]+(?:<[^()]*>)?)", name)
    return m.group(1) if m else name[:60]


def load(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((short(r["Name"]), int(r["Calls"]), int(r["TotalDurationNs"]) / 1e6, float(r["AverageNs"]) / 1e3))
    return rows


if __name__ == "__main__":
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    rows = load(sys.argv[1])
    tot = sum(r[2] for r in rows)
    print(f"total {tot:.2f} ms over {sum(r[1] for r in rows)} launches")
    for n, c, ms, avg in sorted(rows, key=lambda r: -r[2])[:top]:
        print(f"{n[:60]:60s} {c:6d} {ms:9.3f} ms {avg:9.1f} us")
