#!/bin/bash
# GPU box session: parity tests, smoke, the bench workloads, and a rocprofv3 kernel-trace summary.
# usage: tools/gpu_check.sh TAG [pytest-args...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-run}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "$@" > "$OUT/pytest_gpu.log" 2>&1 || { echo PYTEST_FAIL; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
timeout -k 10 600 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo SMOKE_FAIL; tail -20 "$OUT/smoke.log"; exit 1; }
timeout -k 10 600 python bench.py --steps 5 --warmup 2 --stages > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo BENCH_FAIL; tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
for W in C5 C4; do
  timeout -k 10 600 python bench.py --workload $W --steps 5 --warmup 2 --no-cpu-baseline --no-fm --stages > "$OUT/bench_$W.json" 2> "$OUT/bench_$W.err" || { echo BENCH_${W}_FAIL; tail -20 "$OUT/bench_$W.err"; exit 1; }
  cat "$OUT/bench_$W.json"
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > "$OUT/bench_prof.json" 2> "$OUT/prof_stderr.log" || { echo PROF_FAIL; exit 1; }
echo ALL_OK
