#!/bin/bash
# GPU box: one C4 shard at 1/8 and all of the host cores, then the full-size
# C3 CPU comparator (host only)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-cmp}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/c4_shard.py "$OUT/c4_shard.json" 2 16 > "$OUT/c4_shard.log" 2>&1 || { echo SHARD_FAIL; tail -20 "$OUT/c4_shard.log"; exit 1; }
tail -4 "$OUT/c4_shard.log"
timeout -k 10 1000 python -u tools/cpu_c3.py "$OUT/cpu_c3.json" --cap 700 > "$OUT/cpu_c3.log" 2>&1 || { echo CPU_FAIL; tail -20 "$OUT/cpu_c3.log"; exit 1; }
tail -2 "$OUT/cpu_c3.log"
