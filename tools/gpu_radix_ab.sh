#!/bin/bash
# radix A/B: $VAR (default BWTMI_RADIX32, the 32-bit-key geometry) takes each of $VARIANTS
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-radix_ab}
mkdir -p "$OUT"
export TMPDIR=/tmp
VAR=${VAR:-BWTMI_RADIX32}
for v in ${VARIANTS:-0 1 2 3 4 0}; do
  env $VAR=$v timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-fm > "$OUT/v$v.json" 2> "$OUT/v$v.err" || { echo FAIL $v; tail -5 "$OUT/v$v.err"; exit 1; }
  python - "$OUT/v$v.json" $v <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k=d["kernels_ms_per_step"]
print("variant",sys.argv[2],"value",round(d["value"],1),"kv8",k.get("radix_scatter_kv8"),"kv12",k.get("radix_scatter_kv12"),"rank0",k.get("dna_rank0"),"hist",k.get("radix_hist"),"index",d["stage_ms_last_step"]["index"],"sha",d["golden"]["match"])
PY
done
