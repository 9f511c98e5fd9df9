#!/bin/bash
# r03t: restored tree -- GPU suite, C3 line with stage stats, W=8 shard step with stage stats
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r03t}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { echo PYTEST_FAIL; tail -40 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for i in 1 2; do
  (export BWTMI_STATS=1; timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-fm --no-cli > "$OUT/bench_C3_$i.json" 2> "$OUT/bench_C3_$i.err") || { echo BENCH_FAIL; tail -5 "$OUT/bench_C3_$i.err"; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/bench_C3_$i.json').read().strip().splitlines()[-1]); print('C3', d['value'], d['calls_ms_per_step'], d['golden']['match'])"
done
(export C4_SHARD_WORLDS=8 BWTMI_STATS=1; timeout -k 10 300 python -u tools/c4_shard.py "$OUT/c4_shards.json" 16 > "$OUT/c4_shards.log" 2>&1) || { echo SHARD_FAIL; tail -20 "$OUT/c4_shards.log"; exit 1; }
grep -h '"step_ms"' "$OUT/c4_shards.log" | cut -c1-260
echo ALL_OK
