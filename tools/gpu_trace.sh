#!/bin/bash
# GPU box: per-launch timeline of C3 steps (BWTMI_KTRACE: name, ms, idle gap
# since the previous launch on the stream) and a rocprofv3 kernel-stats run
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-trace}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
BWTMI_KTRACE=$OUT/ktrace.txt timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-fm ${BENCH_ARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo BENCH_FAIL; tail -20 "$OUT/bench.err"; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'],d['golden']['match'],d['calls_ms_per_step'],d['stage_ms_last_step'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-fm ${BENCH_ARGS:-} > "$OUT/bench_prof.json" 2> "$OUT/prof_stderr.log" || { echo PROF_FAIL; tail -5 "$OUT/prof_stderr.log"; exit 1; }
echo TRACE_OK
