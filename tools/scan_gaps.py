"""Device idle time inside the scan call: for the last `bwtmi:scan` roctx range
of a rocprofv3 --marker-trace --kernel-trace run, the kernels that ran in it
in start order, the idle gaps between them (the device waiting for the host:
launch latency, host reads of counts) and the largest gaps with the kernel
before each.
usage: python tools/scan_gaps.py marker_api_trace.csv kernel_trace.csv [range]"""
import csv
import sys


def main():
    want = sys.argv[3] if len(sys.argv) > 3 else "bwtmi:scan"
    ranges = []
    with open(sys.argv[1]) as f:
        for r in csv.DictReader(f):
            msg = r.get("Function") or r.get("Message") or r.get("Marker_Message") or ""
            if msg == want:
                ranges.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    if not ranges:
        print("no range", want)
        return
    a, b = sorted(ranges)[-1]
    kern = []
    with open(sys.argv[2]) as f:
        for r in csv.DictReader(f):
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            if a <= s < b:
                kern.append((s, e, r.get("Kernel_Name", "?")[:60]))
    kern.sort()
    busy = sum(e - s for s, e, _ in kern)
    gaps = []
    prev_end, prev_name = a, "(range start)"
    for s, e, nm in kern:
        if s > prev_end:
            gaps.append((s - prev_end, prev_name, nm))
        if e > prev_end:
            prev_end, prev_name = e, nm
    tail = b - prev_end
    print(f"range {want}: {(b - a) / 1e3:.1f} us, {len(kern)} kernels, busy {busy / 1e3:.1f} us, "
          f"idle between kernels {sum(g for g, _, _ in gaps) / 1e3:.1f} us, after the last {tail / 1e3:.1f} us")
    for g, p, n in sorted(gaps, reverse=True)[:15]:
        print(f"  {g / 1e3:8.1f} us  after {p}  before {n}")


if __name__ == "__main__":
    main()
