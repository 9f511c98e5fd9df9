#!/bin/bash
# r03x: LDS tile put after the 16-bit position order; per-chromosome record lists filled in
# parallel (multi-contig write) -- GPU suite, rocprofv3 stats + PMC of the C3 step, C4 line,
# shard steps of worlds 8/4/2, the default bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r03x}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { echo PYTEST_FAIL; tail -40 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
bash tools/gpu_prof_r03.sh "${1:-r03x}" || exit 1
python3 -c "import json; d=json.load(open('$OUT/pmc_traffic.json'))['kernels']; [print(k, v) for k, v in d.items() if 'put' in k or 'scatter' in k]"
(export BWTMI_STATS=1; timeout -k 10 300 python bench.py --workload C4 --steps 10 --warmup 2 --no-cpu-baseline --no-fm --no-cli > "$OUT/bench_C4.json" 2> "$OUT/bench_C4.err") || { echo C4_FAIL; tail -5 "$OUT/bench_C4.err"; exit 1; }
python -c "import json; d=json.loads(open('$OUT/bench_C4.json').read().strip().splitlines()[-1]); print('C4', d['value'], d['calls_ms_per_step'], d['golden']['match'])"
(export C4_SHARD_WORLDS=8,4,2 BWTMI_STATS=1; timeout -k 10 400 python -u tools/c4_shard.py "$OUT/c4_shards.json" 16 > "$OUT/c4_shards.log" 2>&1) || { echo SHARD_FAIL; tail -20 "$OUT/c4_shards.log"; exit 1; }
grep -h '"step_ms"' "$OUT/c4_shards.log" | cut -c1-330
timeout -k 10 400 python bench.py --pmc-summary "$OUT/pmc_traffic.json" > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" || { echo BENCH_FAIL; tail -5 "$OUT/bench_default.err"; exit 1; }
python -c "import json; d=json.loads(open('$OUT/bench_default.json').read().strip().splitlines()[-1]); k=d['kernels_ms_per_step']; print(d['value'], d['calls_ms_per_step'], d['golden']['match'], d['roofline'], k.get('dna_rank_put'), k.get('radix_partition_kv8'), d['stage_ms_last_step'])"
echo ALL_OK
