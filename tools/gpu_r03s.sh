#!/bin/bash
# r03s: writer speedups, collapse chunks from the fold, one-word screened hits --
# the GPU suite, C3 lines, C5 line, 8-rank C4 shard step
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r03s}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_load.py -x -v --timeout 250 --timeout-method thread > "$OUT/pytest_new.log" 2>&1 || { echo NEW_FAIL; tail -40 "$OUT/pytest_new.log"; exit 1; }
tail -1 "$OUT/pytest_new.log"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { echo PYTEST_FAIL; tail -40 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for i in 1 2 3 4; do
  spin=1; [ $((i % 2)) = 0 ] && spin=0
  (export BWTMI_STATS=1 BWTMI_SPIN_SCAN=$spin; timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-fm --no-cli > "$OUT/bench_C3_$i.json" 2> "$OUT/bench_C3_$i.err") || { echo BENCH_FAIL; tail -5 "$OUT/bench_C3_$i.err"; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/bench_C3_$i.json').read().strip().splitlines()[-1]); print('C3 spin=$spin', d['value'], d['calls_ms_per_step'], d['golden']['match'])"
done
(export BWTMI_STATS=1; timeout -k 10 300 python bench.py --workload C5 --steps 10 --warmup 2 --no-cpu-baseline --no-fm --no-cli > "$OUT/bench_C5.json" 2> "$OUT/bench_C5.err") || { echo C5_FAIL; tail -5 "$OUT/bench_C5.err"; exit 1; }
python -c "import json; d=json.loads(open('$OUT/bench_C5.json').read().strip().splitlines()[-1]); print('C5', d['value'], d['calls_ms_per_step'], d['golden']['match'])"
(export C4_SHARD_WORLDS=8; timeout -k 10 300 python -u tools/c4_shard.py "$OUT/c4_shards.json" 16 > "$OUT/c4_shards.log" 2>&1) || { echo SHARD_FAIL; tail -20 "$OUT/c4_shards.log"; exit 1; }
grep -h '"step_ms"' "$OUT/c4_shards.log" | cut -c1-260
echo ALL_OK
