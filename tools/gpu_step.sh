#!/bin/bash
# host-stage breakdown of the bench step on the GPU box (BWTMI_STATS=1, then =2 counters)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-step}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
BWTMI_STATS=1 timeout -k 10 300 python -u tools/step_profile.py 4 > "$OUT/step.log" 2>&1 || { echo STEP_FAIL; tail -20 "$OUT/step.log"; exit 1; }
grep -v "^  m~" "$OUT/step.log" | tail -24
BWTMI_STATS=2 timeout -k 10 300 python -u tools/step_profile.py 2 > "$OUT/step2.log" 2>&1 || { echo STEP2_FAIL; tail -20 "$OUT/step2.log"; exit 1; }
tail -40 "$OUT/step2.log"
