#!/bin/bash
# r03p: device FASTA load with per-piece image copies and plain tails --
# its parity tests, the GPU suite, and an alternating C3 A/B (device / host load)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r03p}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_load.py -x -v --timeout 200 --timeout-method thread > "$OUT/pytest_new.log" 2>&1 || { echo NEW_FAIL; tail -40 "$OUT/pytest_new.log"; exit 1; }
tail -1 "$OUT/pytest_new.log"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { echo PYTEST_FAIL; tail -40 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
i=0
for mode in dev host dev host dev host; do
  i=$((i+1))
  flag=""; [ $mode = host ] && flag="--host-load"
  (export BWTMI_STATS=1; timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-fm --no-cli $flag > "$OUT/bench_C3_${mode}_$i.json" 2> "$OUT/bench_C3_${mode}_$i.err") || { echo BENCH_FAIL $mode; tail -5 "$OUT/bench_C3_${mode}_$i.err"; exit 1; }
  python -c "import json,sys; d=json.loads(open('$OUT/bench_C3_${mode}_$i.json').read().strip().splitlines()[-1]); print('$mode', d['value'], d['calls_ms_per_step'], d['golden']['match'])"
done
echo ALL_OK
