#!/bin/bash
# r03v: C4 on one GPU and the shard steps of worlds 2/4/8 (stage stats)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r03v}
mkdir -p "$OUT"
export TMPDIR=/tmp
(export BWTMI_STATS=1; timeout -k 10 300 python bench.py --workload C4 --steps 10 --warmup 2 --no-cpu-baseline --no-fm --no-cli > "$OUT/bench_C4.json" 2> "$OUT/bench_C4.err") || { echo C4_FAIL; tail -5 "$OUT/bench_C4.err"; exit 1; }
python -c "import json; d=json.loads(open('$OUT/bench_C4.json').read().strip().splitlines()[-1]); print('C4', d['value'], d['calls_ms_per_step'], d['golden']['match'])"
(export C4_SHARD_WORLDS=8,4,2 BWTMI_STATS=1; timeout -k 10 400 python -u tools/c4_shard.py "$OUT/c4_shards.json" 16 > "$OUT/c4_shards.log" 2>&1) || { echo SHARD_FAIL; tail -20 "$OUT/c4_shards.log"; exit 1; }
grep -h '"step_ms"' "$OUT/c4_shards.log" | cut -c1-330
echo ALL_OK
