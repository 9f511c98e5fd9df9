#!/bin/bash
# host-thread count A/B of the bench step (tools/step_profile.py), same box
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-threads_ab}
mkdir -p "$OUT"
export TMPDIR=/tmp
for t in 16 15 14 16 12; do
  STEP_THREADS=$t timeout -k 10 300 python -u tools/step_profile.py 5 > "$OUT/t$t.log" 2>&1 || { echo FAIL; tail -5 "$OUT/t$t.log"; exit 1; }
  echo "threads $t"; tail -3 "$OUT/t$t.log" | cut -c1-120
done
