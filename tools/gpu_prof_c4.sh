#!/bin/bash
# rocprofv3 kernel trace of the C4 bench (8 contigs on one GPU) and the C3 host-stage counters
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-profc4}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 bench.py --workload C4 --steps 1 --warmup 1 --no-cpu-baseline --no-fm > "$OUT/bench_prof.json" 2> "$OUT/prof_stderr.log" || { echo PROF_FAIL; tail -5 "$OUT/prof_stderr.log"; exit 1; }
BWTMI_STATS=2 timeout -k 10 300 python -u tools/step_profile.py 3 > "$OUT/step.log" 2>&1 || { echo STEP_FAIL; tail -20 "$OUT/step.log"; exit 1; }
tail -30 "$OUT/step.log"
echo PROF_OK
