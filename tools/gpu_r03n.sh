#!/bin/bash
# r03n: per-launch device timeline of the C3 step (BWTMI_KTRACE)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r03n}
mkdir -p "$OUT"
export TMPDIR=/tmp
(export BWTMI_KTRACE="$OUT/c3_ktrace.txt" BWTMI_STATS=1; timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-fm --no-cli > "$OUT/c3_traced.json" 2> "$OUT/c3_traced.err") || { echo C3TRACE_FAIL; tail -20 "$OUT/c3_traced.err"; exit 1; }
echo ALL_OK
