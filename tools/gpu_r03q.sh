#!/bin/bash
# r03q: split loader with device placement -- its parity tests, the GPU suite,
# the C4 line on one GPU, a 2-rank self-launched C4 rehearsal (one GPU, host
# transport), and the 8-rank C4 shard step with device / host load
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r03q}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_load.py -x -v --timeout 200 --timeout-method thread > "$OUT/pytest_new.log" 2>&1 || { echo NEW_FAIL; tail -40 "$OUT/pytest_new.log"; exit 1; }
tail -1 "$OUT/pytest_new.log"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { echo PYTEST_FAIL; tail -40 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
(export BWTMI_STATS=1; timeout -k 10 300 python bench.py --workload C4 --steps 10 --warmup 2 --no-cpu-baseline --no-fm --no-cli > "$OUT/bench_C4.json" 2> "$OUT/bench_C4.err") || { echo C4_FAIL; tail -5 "$OUT/bench_C4.err"; exit 1; }
python -c "import json; d=json.loads(open('$OUT/bench_C4.json').read().strip().splitlines()[-1]); print('C4', d['value'], d['calls_ms_per_step'], d['golden']['match'])"
(export BWTMI_BENCH_GLOO=1; timeout -k 10 300 python bench.py --gpus 2 --steps 5 --warmup 1 --no-cpu-baseline --no-fm --no-cli > "$OUT/bench_C4_2rank.json" 2> "$OUT/bench_C4_2rank.err") || { echo R2_FAIL; tail -20 "$OUT/bench_C4_2rank.err"; exit 1; }
python -c "import json; d=json.loads(open('$OUT/bench_C4_2rank.json').read().strip().splitlines()[-1]); print('C4x2', d['n_gpus'], d['value'], d['golden']['match'])"
for dl in 1 0; do
  (export C4_SHARD_WORLDS=8 C4_SHARD_DEVLOAD=$dl BWTMI_STATS=1; timeout -k 10 300 python -u tools/c4_shard.py "$OUT/c4_shards_dl$dl.json" 16 > "$OUT/c4_shards_dl$dl.log" 2>&1) || { echo SHARD_FAIL; tail -20 "$OUT/c4_shards_dl$dl.log"; exit 1; }
  grep -h '"step_ms"' "$OUT/c4_shards_dl$dl.log" | cut -c1-300
done
echo ALL_OK
