#!/bin/bash
# r03ab: pool spin 0 / 10 us on the C3 line, 3 runs each, alternating on one box
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r03ab}
mkdir -p "$OUT"
export TMPDIR=/tmp
for i in 1 2 3 4 5 6; do
  spin=10; [ $((i % 2)) = 1 ] && spin=0
  (export BWTMI_POOL_SPIN_US=$spin; timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-fm --no-cli > "$OUT/bench_C3_$i.json" 2> "$OUT/bench_C3_$i.err") || { echo BENCH_FAIL; tail -5 "$OUT/bench_C3_$i.err"; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/bench_C3_$i.json').read().strip().splitlines()[-1]); print('C3 spin=$spin', d['value'], d['calls_ms_per_step'], d['golden']['match'])"
done
echo ALL_OK
