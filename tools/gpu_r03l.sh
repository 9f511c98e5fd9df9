#!/bin/bash
# r03l: re-entry check of the restored tree -- GPU suite, default bench line, C5 line
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r03l}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { echo PYTEST_FAIL; tail -40 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 300 python bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" || { echo BENCH_FAIL; tail -5 "$OUT/bench_default.err"; exit 1; }
(export BWTMI_STATS=1; timeout -k 10 300 python bench.py --workload C5 --steps 10 --warmup 2 --no-cpu-baseline --no-fm --no-cli > "$OUT/bench_C5.json" 2> "$OUT/bench_C5.err") || { echo BENCH_FAIL C5; tail -5 "$OUT/bench_C5.err"; exit 1; }
echo ALL_OK
