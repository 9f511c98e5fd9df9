#!/bin/bash
# r03e: GPU suite; segmented nested levels (one launch) vs per-level launches on
# C3 / C4 and the 8-rank C4 shard step
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r03e}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { echo PYTEST_FAIL; tail -40 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for seg in 1 0; do
  for w in C3 C4; do
    (export BWTMI_SEG_LEVELS=$seg; timeout -k 10 300 python bench.py --workload $w --steps 10 --warmup 2 --no-cpu-baseline --no-fm --no-cli > "$OUT/bench_${w}_seg$seg.json" 2> "$OUT/bench_${w}_seg$seg.err") || { echo BENCH_FAIL $w $seg; tail -5 "$OUT/bench_${w}_seg$seg.err"; exit 1; }
  done
done
echo BENCH_OK
for seg in 1 0; do
  (export BWTMI_SEG_LEVELS=$seg C4_SHARD_WORLDS=8; timeout -k 10 300 python -u tools/c4_shard.py "$OUT/c4_shards_seg$seg.json" 16 > "$OUT/c4_shards_seg$seg.log" 2>&1) || { echo SHARD_FAIL; tail -20 "$OUT/c4_shards_seg$seg.log"; exit 1; }
done
echo ALL_OK
