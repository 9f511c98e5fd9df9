#!/bin/bash
# GPU box: FM / index parity tests, then the bench line with the FM query timing
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-fm}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "index or dna or backward or lcp or library or tier3 or smoke or locate or kmer" > "$OUT/pytest_gpu.log" 2>&1 || { echo PYTEST_FAIL; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
timeout -k 10 600 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo BENCH_FAIL; tail -20 "$OUT/bench.err"; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print('C3',d['value'],d['fm_all_motifs_1_10'],d['roofline'])"
