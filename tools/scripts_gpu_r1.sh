#!/bin/bash
# round-1 GPU session: smoke -> GPU parity tests -> bench (each step bounded)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; exit 1; }
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; exit 1; }
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --stages --contig-bp 10000000 > gpurun_out/bench10m.json 2> gpurun_out/bench10m.err || { echo BENCH10_FAIL; exit 1; }
timeout -k 10 600 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --stages > gpurun_out/bench1.json 2> gpurun_out/bench1.err || { echo BENCH_FAIL; exit 1; }
echo ALL_OK
