#!/bin/bash
# SQ counters per dispatch (one rocprofv3 --pmc pass) for the scan kernels.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-sq}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d "$OUT/sq" -o pmc -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-fm --no-index > "$OUT/sq.json" 2> "$OUT/sq.err" || { echo SQ_FAIL; tail -5 "$OUT/sq.err"; exit 1; }
python3 - "$OUT/sq" <<'PY'
import csv, glob, os, sys
f = glob.glob(os.path.join(sys.argv[1], "**", "*counter_collection*.csv"), recursive=True)[0]
rows = list(csv.DictReader(open(f)))
keep = ("k_runs", "k_level", "k_scatter", "k_period")
agg = {}
for r in rows:
    n = r["Kernel_Name"]
    k = next((x for x in keep if x in n), None)
    if not k: continue
    agg.setdefault((k, r["Dispatch_Id"]), {})[r["Counter_Name"]] = float(r["Counter_Value"])
tot = {}
for (k, d), c in agg.items():
    t = tot.setdefault(k, {})
    for cn, v in c.items(): t[cn] = t.get(cn, 0) + v
for k, c in tot.items(): print(k, {a: f"{b:.3g}" for a, b in sorted(c.items())})
PY
