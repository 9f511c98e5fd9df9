#!/bin/bash
# host-stage breakdown of the C3 / C5 steps (BWTMI_STATS=1 on stderr)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r03g}
mkdir -p "$OUT"
export TMPDIR=/tmp
for w in C3 C5; do
  (export BWTMI_STATS=1; timeout -k 10 300 python bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline --no-fm --no-cli > "$OUT/stats_$w.json" 2> "$OUT/stats_$w.err") || { echo FAIL $w; tail -5 "$OUT/stats_$w.err"; exit 1; }
done
echo ALL_OK
