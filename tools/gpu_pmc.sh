#!/bin/bash
# HBM traffic per kernel: two separate rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE
# cannot share a pass on gfx950), then tools/pmc_traffic.py.
# usage: tools/gpu_pmc.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-pmc}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o pmc -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > "$OUT/fetch.json" 2> "$OUT/fetch.err" || { echo FETCH_FAIL; tail -5 "$OUT/fetch.err"; exit 1; }
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o pmc -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > "$OUT/write.json" 2> "$OUT/write.err" || { echo WRITE_FAIL; tail -5 "$OUT/write.err"; exit 1; }
python3 tools/pmc_traffic.py "$OUT/fetch" "$OUT/write" "$OUT/pmc_traffic.json" && echo PMC_OK
