#!/bin/bash
# Same-box A/B of two library builds on one bench workload, alternating runs
# (box-to-box spread of the host stages is +-10-15 %, so only same-box pairs
# are compared).  usage: tools/ab_bench.sh TAG A_LIB REPS [bench.py args]
# B is the in-tree libbwtmi.so.  Outputs gpurun_out/TAG/ab_{A,B}_k.json
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=$1; ALIB=$2; REPS=$3; shift 3
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for k in $(seq 1 "$REPS"); do
  BWTMI_LIB=$ALIB timeout -k 10 300 python bench.py --no-cpu-baseline --no-fm --no-cli "$@" > "$OUT/ab_A_$k.json" 2> "$OUT/ab_A_$k.err" || { echo A_FAIL; tail -5 "$OUT/ab_A_$k.err"; exit 1; }
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-fm --no-cli "$@" > "$OUT/ab_B_$k.json" 2> "$OUT/ab_B_$k.err" || { echo B_FAIL; tail -5 "$OUT/ab_B_$k.err"; exit 1; }
done
python3 - "$OUT" "$REPS" <<'PY'
import json, sys
out, reps = sys.argv[1], int(sys.argv[2])
for arm in "AB":
    rows = [json.loads(open(f"{out}/ab_{arm}_{k}.json").read().strip().splitlines()[-1]) for k in range(1, reps + 1)]
    print(arm, "Mbp/s", [r["value"] for r in rows], "golden", [r["golden"]["match"] if r["golden"] else None for r in rows])
    keys = rows[0]["calls_ms_per_step"].keys()
    print("  calls", {k: [r["calls_ms_per_step"][k] for r in rows] for k in keys if k in ("scan", "postprocess", "write", "load_fasta")})
PY
