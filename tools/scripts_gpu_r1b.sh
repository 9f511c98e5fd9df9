#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof_r01
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; exit 1; }
timeout -k 10 600 python bench.py --steps 2 --warmup 1 --stages > gpurun_out/bench2.json 2> gpurun_out/bench2.err || { echo BENCH_FAIL; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r01 -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/prof_r01/bench_prof.json 2> gpurun_out/prof_r01/stderr.log || { echo PROF_FAIL; exit 1; }
echo ALL_OK
