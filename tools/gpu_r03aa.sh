#!/bin/bash
# r03aa: final tree -- GPU suite, smoke(), default bench line; short-spin A/B
# (BWTMI_POOL_SPIN_US 0 / 10) on C3 and the W=8 shard step, alternating
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r03aa}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { echo PYTEST_FAIL; tail -40 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > "$OUT/smoke.log" 2>&1 || { echo SMOKE_FAIL; tail -20 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
timeout -k 10 400 python bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" || { echo BENCH_FAIL; tail -5 "$OUT/bench_default.err"; exit 1; }
python -c "import json; d=json.loads(open('$OUT/bench_default.json').read().strip().splitlines()[-1]); print('default', d['value'], d['calls_ms_per_step'], d['golden']['match'], d['roofline']['frac'], d['roofline']['traffic'], d['cpu_baseline']['value'], d.get('cli_drop_in', {}).get('vs_step'))"
for i in 1 2 3 4; do
  spin=10; [ $((i % 2)) = 1 ] && spin=0
  (export BWTMI_POOL_SPIN_US=$spin; timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-fm --no-cli > "$OUT/bench_C3_$i.json" 2> "$OUT/bench_C3_$i.err") || { echo BENCH_FAIL; tail -5 "$OUT/bench_C3_$i.err"; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/bench_C3_$i.json').read().strip().splitlines()[-1]); print('C3 spin=$spin', d['value'], d['calls_ms_per_step'], d['golden']['match'])"
done
for spin in 0 10; do
  (export C4_SHARD_WORLDS=8 BWTMI_POOL_SPIN_US=$spin; timeout -k 10 300 python -u tools/c4_shard.py "$OUT/c4_shards_$spin.json" 16 > "$OUT/c4_shards_$spin.log" 2>&1) || { echo SHARD_FAIL; tail -20 "$OUT/c4_shards_$spin.log"; exit 1; }
  echo "shard spin=$spin"; grep -h '"step_ms"' "$OUT/c4_shards_$spin.log" | cut -c1-110
done
echo ALL_OK
