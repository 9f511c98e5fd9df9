#!/bin/bash
# does live kernel timing (bench.py) slow the host stages?  step profile with and without it
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-kstats_ab}
mkdir -p "$OUT"
export TMPDIR=/tmp
for k in 0 1 0 1; do
  STEP_KSTATS=$k timeout -k 10 300 python -u tools/step_profile.py 6 > "$OUT/k$k.log" 2>&1 || { echo FAIL; tail -5 "$OUT/k$k.log"; exit 1; }
  echo "kstats $k"; tail -3 "$OUT/k$k.log" | cut -c1-110
done
