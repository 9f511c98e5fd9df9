#!/bin/bash
# A/B of the radix pass geometries (BWTMI_RADIX=<items>,<nt>,<split>) on the bench workload.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-radix}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for v in 16,0,1 20,0,1 24,0,1 12,0,1 8,0,1 16,0,0; do
  BWTMI_RADIX=$v timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-fm > "$OUT/bench_$v.json" 2> "$OUT/bench_$v.err" || { echo "FAIL $v"; tail -5 "$OUT/bench_$v.err"; exit 1; }
  python3 -c "
import json,sys; d=json.load(open('$OUT/bench_$v.json')); r=d['roofline']; k=d['kernels_ms_per_step']
print('$v', d['value'], d['output_sha256'][:12], r['kernel'], r['frac'], r['avg_launch_ms'], 'scatter12', k.get('radix_scatter_kv12'), 'hist', k.get('radix_hist'), 'idx', d['stage_ms_last_step']['index'])"
done
