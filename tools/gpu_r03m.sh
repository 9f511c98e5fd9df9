#!/bin/bash
# r03m: host sampler of the C3 step (the fold's recomputes on the host)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r03m}
mkdir -p "$OUT"
export TMPDIR=/tmp
(export BWTMI_STATS=1; timeout -k 10 300 python -u tools/sampler.py "$OUT/samp" 20 > "$OUT/samp.log" 2>&1) || { echo SAMP_FAIL; tail -20 "$OUT/samp.log"; exit 1; }
rm -f "$OUT/samp.raw" "$OUT/samp.raw.chains"
echo ALL_OK
