"""Stage ranges of a rocprofv3 --marker-trace run (roctx "bwtmi:<stage>",
csrc/trace.cpp) with the kernels that ran inside each: per stage the wall ms
of its ranges (summed over calls and threads) and the GPU ms of the kernels
that started inside them.
usage: python tools/stage_ranges.py marker_api_trace.csv kernel_trace.csv"""
import csv
import sys
from collections import defaultdict


def main():
    ranges = []
    with open(sys.argv[1]) as f:
        for r in csv.DictReader(f):
            msg = r.get("Function") or r.get("Message") or r.get("Marker_Message") or ""
            if not msg.startswith("bwtmi"):
                continue
            ranges.append((msg, int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Thread_Id", "")))
    kern = []
    with open(sys.argv[2]) as f:
        for r in csv.DictReader(f):
            kern.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    agg = defaultdict(lambda: [0.0, 0, 0.0, 0])
    for name, a, b, _ in ranges:
        g = agg[name]
        g[0] += (b - a) / 1e6
        g[1] += 1
        for ka, kb in kern:
            if a <= ka < b:
                g[2] += (kb - ka) / 1e6
                g[3] += 1
    print(f"{'range':28s} {'calls':>5s} {'wall ms':>9s} {'kernels':>8s} {'kernel ms':>9s}")
    for name, (w, c, km, kc) in sorted(agg.items(), key=lambda kv: -kv[1][0]):
        print(f"{name:28s} {c:5d} {w:9.2f} {kc:8d} {km:9.2f}")


if __name__ == "__main__":
    main()
