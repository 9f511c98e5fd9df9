#!/bin/bash
# r03j: device DP recomputes of the merge fold -- parity tests, GPU suite, and
# A/B (BWTMI_POST_DEVICE=1/0) on C3, C5 and the 8-rank C4 shard step
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r03j}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_recompute.py -x -v --timeout 120 --timeout-method thread > "$OUT/pytest_rc.log" 2>&1 || { echo RC_FAIL; tail -40 "$OUT/pytest_rc.log"; exit 1; }
tail -1 "$OUT/pytest_rc.log"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { echo PYTEST_FAIL; tail -40 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for pd in 1 0; do
  for w in C3 C5; do
    (export BWTMI_POST_DEVICE=$pd BWTMI_STATS=1; timeout -k 10 300 python bench.py --workload $w --steps 10 --warmup 2 --no-cpu-baseline --no-fm --no-cli > "$OUT/bench_${w}_pd$pd.json" 2> "$OUT/bench_${w}_pd$pd.err") || { echo BENCH_FAIL $w $pd; tail -5 "$OUT/bench_${w}_pd$pd.err"; exit 1; }
  done
done
echo BENCH_OK
for pd in 1 0; do
  (export BWTMI_POST_DEVICE=$pd C4_SHARD_WORLDS=8; timeout -k 10 300 python -u tools/c4_shard.py "$OUT/c4_shards_pd$pd.json" 16 > "$OUT/c4_shards_pd$pd.log" 2>&1) || { echo SHARD_FAIL; tail -20 "$OUT/c4_shards_pd$pd.log"; exit 1; }
done
echo ALL_OK
