#!/bin/bash
# radix scatter geometry A/B: BWTMI_RADIX selects <block>x<items>; bench line per variant
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-radix_ab}
mkdir -p "$OUT"
export TMPDIR=/tmp
for v in ${VARIANTS:-0 3 5 6 7 8 3}; do
  BWTMI_RADIX=$v timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > "$OUT/v$v.json" 2> "$OUT/v$v.err" || { echo FAIL $v; tail -5 "$OUT/v$v.err"; exit 1; }
  python - "$OUT/v$v.json" $v <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r=d.get("roofline",{})
print("variant",sys.argv[2],"value",round(d["value"],1),"ms",round(d["ms_per_step"],2),"frac",r.get("frac"),"achieved",r.get("achieved"),"sha",str(d.get("output_sha256",""))[:16])
PY
done
