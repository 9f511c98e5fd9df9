#!/bin/bash
# r03u: spin-then-block worker pool A/B (BWTMI_POOL_SPIN_US=0 is the blocking hand-off):
# C3 lines and the W=8 shard step, alternating; the GPU suite first (radix scatter at 3 workgroups
# per CU, blocked vector chunk scans)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r03u}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { echo PYTEST_FAIL; tail -40 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for i in 1 2 3 4; do
  spin=60; [ $((i % 2)) = 1 ] && spin=0
  (export BWTMI_STATS=1 BWTMI_POOL_SPIN_US=$spin; timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-fm --no-cli > "$OUT/bench_C3_$i.json" 2> "$OUT/bench_C3_$i.err") || { echo BENCH_FAIL; tail -5 "$OUT/bench_C3_$i.err"; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/bench_C3_$i.json').read().strip().splitlines()[-1]); print('C3 spin=$spin', d['value'], d['calls_ms_per_step'], d['golden']['match'], d['roofline']['frac'], d['roofline']['avg_launch_ms'], d['kernels_ms_per_step'].get('radix_partition_kv8'), d.get('device_ms_per_step'))"
done
for i in 1 2; do
  spin=60; [ $((i % 2)) = 1 ] && spin=0
  (export C4_SHARD_WORLDS=8 BWTMI_STATS=1 BWTMI_POOL_SPIN_US=$spin; timeout -k 10 300 python -u tools/c4_shard.py "$OUT/c4_shards_$i.json" 16 > "$OUT/c4_shards_$i.log" 2>&1) || { echo SHARD_FAIL; tail -20 "$OUT/c4_shards_$i.log"; exit 1; }
  echo "shard spin=$spin"; grep -h '"step_ms"' "$OUT/c4_shards_$i.log" | cut -c1-200
done
echo ALL_OK
