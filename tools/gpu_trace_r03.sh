#!/bin/bash
# per-launch device timelines (BWTMI_KTRACE: kernel ms and the device gap before it)
# of the 8-rank C4 shard step and of the C3 step
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r03d}
mkdir -p "$OUT"
export TMPDIR=/tmp
(export BWTMI_KTRACE="$OUT/c4_ktrace.txt" C4_SHARD_WORLDS=8; timeout -k 10 300 python -u tools/c4_shard.py "$OUT/c4_shards_traced.json" 16 > "$OUT/c4_shards_traced.log" 2>&1) || { echo TRACE_FAIL; tail -20 "$OUT/c4_shards_traced.log"; exit 1; }
(export BWTMI_KTRACE="$OUT/c3_ktrace.txt"; timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-fm --no-cli > "$OUT/c3_traced.json" 2> "$OUT/c3_traced.err") || { echo C3TRACE_FAIL; tail -20 "$OUT/c3_traced.err"; exit 1; }
echo ALL_OK
