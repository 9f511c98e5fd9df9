#!/bin/bash
# r03c: GPU suite, C3/C5/C4 bench lines, library kernels (HIP events +
# rocprofv3 stats), the 8-rank C4 shard step with a per-launch trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r03c}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { echo PYTEST_FAIL; tail -40 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for w in C3 C5 C4 C3; do
  timeout -k 10 300 python bench.py --workload $w --steps 10 --warmup 2 --no-cpu-baseline --no-fm > "$OUT/bench_$w.json" 2> "$OUT/bench_$w.err" || { echo BENCH_FAIL $w; tail -5 "$OUT/bench_$w.err"; exit 1; }
done
echo BENCH_OK
timeout -k 10 300 python -u tools/lib_kernels.py "$OUT/lib_kernels.json" 999000 1e7 > "$OUT/lib_kernels.log" 2>&1 || { echo LIB_FAIL; tail -20 "$OUT/lib_kernels.log"; exit 1; }
echo LIB_OK
(export BWTMI_STATS=1 C4_SHARD_WORLDS=8; timeout -k 10 300 python -u tools/c4_shard.py "$OUT/c4_shards.json" 16 > "$OUT/c4_shards.log" 2>&1) || { echo SHARD_FAIL; tail -20 "$OUT/c4_shards.log"; exit 1; }
(export BWTMI_KTRACE="$OUT/c4_ktrace.txt" C4_SHARD_WORLDS=8; timeout -k 10 300 python -u tools/c4_shard.py "$OUT/c4_shards_traced.json" 16 > "$OUT/c4_shards_traced.log" 2>&1) || { echo TRACE_FAIL; tail -20 "$OUT/c4_shards_traced.log"; exit 1; }
echo ALL_OK
