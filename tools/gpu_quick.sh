#!/bin/bash
# GPU box: parity tests, C3 + C4 bench lines, host-stage sampling profile
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-quick}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "$@" > "$OUT/pytest_gpu.log" 2>&1 || { echo PYTEST_FAIL; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
timeout -k 10 600 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-fm > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo BENCH_FAIL; tail -20 "$OUT/bench.err"; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print('C3',d['value'],d['ms_per_step'],d['golden']['match'],d['calls_ms_per_step'],d['stage_ms_last_step'],list(d['kernels_ms_per_step'].items())[:10])"
timeout -k 10 600 python bench.py --workload C4 --steps 5 --warmup 2 --no-cpu-baseline --no-fm > "$OUT/bench_C4.json" 2> "$OUT/bench_C4.err" || { echo BENCH_C4_FAIL; tail -20 "$OUT/bench_C4.err"; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench_C4.json'));print('C4',d['value'],d['ms_per_step'],d['golden']['match'],d['calls_ms_per_step'],list(d['kernels_ms_per_step'].items())[:8])"
timeout -k 10 300 python -u tools/sampler.py "$OUT/sampler" 4 > "$OUT/sampler.out" 2>&1 || { echo SAMPLER_FAIL; tail -20 "$OUT/sampler.out"; exit 1; }
head -45 "$OUT/sampler.out"
echo QUICK_OK
