"""Per-kernel HBM traffic from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE).

usage: python tools/pmc_traffic.py FETCH_DIR WRITE_DIR OUT.json

Each DIR holds the csv output of one pass (``rocprofv3 --pmc FETCH_SIZE
--output-format csv -d DIR -o pmc -- python3 bench.py ...``).  Counters are
per dispatch, in KiB.  gfx950 correction (MI355X_MICROARCH.md, HBM): FETCH_SIZE
tallies 128-B read requests at 64 B, so reads are counted twice:
hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.
"""
import csv
import glob
import json
import os
import re
import sys


def short(name: str) -> str:
    m = re.search(r"::(k_[A-Za-z0-9_]+)", name)
    s = m.group(1) if m else name.split("(")[0].strip()
    # type template arguments (k_scatter<key, value, ...>: kv8 = <u32,u32>, kv12 = <u64,u32>)
    ts = re.findall(r"(unsigned int|unsigned long|unsigned short|unsigned char)",
                    name.replace("(anonymous namespace)", "").split("(")[0])
    if ts:
        s += "<" + ",".join({"unsigned int": "u32", "unsigned long": "u64", "unsigned short": "u16", "unsigned char": "u8"}[t]
                            for t in ts[:2]) + ">"
    return s


def load(d: str, counter: str):
    files = glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection csv under {d}")
    tot, n = {}, {}
    for f in files:
        with open(f, newline="") as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                k = short(row.get("Kernel_Name", ""))
                tot[k] = tot.get(k, 0.0) + float(row["Counter_Value"])
                n[k] = n.get(k, 0) + 1
    return tot, n


def main(argv):
    fdir, wdir, out = argv[1:4]
    ft, fn = load(fdir, "FETCH_SIZE")
    wt, wn = load(wdir, "WRITE_SIZE")
    res = {}
    for k in sorted(set(ft) | set(wt)):
        d = max(fn.get(k, 0), wn.get(k, 0))
        f_kib = ft.get(k, 0.0) / max(fn.get(k, 1), 1)
        w_kib = wt.get(k, 0.0) / max(wn.get(k, 1), 1)
        res[k] = {"dispatches": d, "fetch_kib_per_launch": round(f_kib, 1),
                  "write_kib_per_launch": round(w_kib, 1),
                  "hbm_bytes_per_launch": round((2.0 * f_kib + w_kib) * 1024.0)}
    with open(out, "w") as fh:
        json.dump({"correction": "hbm_bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE "
                                 "counts 128-B reads at 64 B)", "kernels": res}, fh, indent=1, sort_keys=True)
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv))
