#!/bin/bash
# r03o: device FASTA load + sampled long-L strict scan -- their parity tests,
# the GPU suite, and the C3 line A/B (device/host load, sampled/dense k_runs)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r03o}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_load.py tests/test_gpu.py -k "load or strict_scan" -x -v --timeout 200 --timeout-method thread > "$OUT/pytest_new.log" 2>&1 || { echo NEW_FAIL; tail -40 "$OUT/pytest_new.log"; exit 1; }
tail -1 "$OUT/pytest_new.log"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { echo PYTEST_FAIL; tail -40 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for mode in new hostdense devdense new hostdense; do
  flag=""; [ $mode = hostdense ] && flag="--host-load"
  dense=0; [ $mode != new ] && dense=1
  (export BWTMI_STATS=1 BWTMI_RUNS_DENSE=$dense; timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-fm --no-cli $flag > "$OUT/bench_C3_$mode.json" 2> "$OUT/bench_C3_$mode.err") || { echo BENCH_FAIL $mode; tail -5 "$OUT/bench_C3_$mode.err"; exit 1; }
  python -c "import json,sys; d=json.loads(open('$OUT/bench_C3_$mode.json').read().strip().splitlines()[-1]); print('$mode', d['value'], d['calls_ms_per_step'], d['golden']['match'], {k:v for k,v in d['kernels_ms_per_step'].items() if 'runs' in k or 'fa_' in k})"
done
echo ALL_OK
