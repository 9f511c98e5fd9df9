#!/bin/bash
# r03r: rocprofv3 stats + PMC passes of the current C3 step, then the default bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r03r}
bash tools/gpu_prof_r03.sh "${1:-r03r}" || exit 1
timeout -k 10 400 python bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" || { echo BENCH_FAIL; tail -5 "$OUT/bench_default.err"; exit 1; }
python -c "import json; d=json.loads(open('$OUT/bench_default.json').read().strip().splitlines()[-1]); print(d['value'], d['calls_ms_per_step'], d['golden']['match'], d['roofline'], d.get('cli'))"
echo ALL_OK
