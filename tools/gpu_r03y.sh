#!/bin/bash
# r03y: per-Mbp host cost against contig size -- single-contig bench steps of 12.5/25/50 Mbp
# (stage stats), host sampler of the 12.5 Mbp step; the cgroup CPU quota and its throttle
# counters around each run
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r03y}
mkdir -p "$OUT"
export TMPDIR=/tmp
cat /sys/fs/cgroup/cpu.max 2>/dev/null; cat /sys/fs/cgroup/cpu.stat 2>/dev/null | grep -i thrott
for bp in 12500000 25000000 50000000 100000000; do
  (export BWTMI_STATS=1; timeout -k 10 300 python bench.py --contig-bp $bp --steps 10 --warmup 2 --no-cpu-baseline --no-fm --no-cli > "$OUT/bench_$bp.json" 2> "$OUT/bench_$bp.err") || { echo BENCH_FAIL; tail -5 "$OUT/bench_$bp.err"; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/bench_$bp.json').read().strip().splitlines()[-1]); print('$bp', d['value'], d['ms_per_step'], d['calls_ms_per_step'])"
  cat /sys/fs/cgroup/cpu.stat 2>/dev/null | grep -i thrott | tr '\n' ' '; echo
done
(export C4_SHARD_WORLDS=8; timeout -k 10 300 python -u tools/c4_shard.py "$OUT/c4_shards.json" 16 > "$OUT/c4_shards.log" 2>&1) || { echo SHARD_FAIL; tail -20 "$OUT/c4_shards.log"; exit 1; }
grep -h '"step_ms"' "$OUT/c4_shards.log" | cut -c1-120
cat /sys/fs/cgroup/cpu.stat 2>/dev/null | grep -i thrott | tr '\n' ' '; echo
g++ -O2 -shared -fPIC tools/sampler.cpp -o tools/libsampler.so || exit 1
timeout -k 10 300 python tools/sampler.py "$OUT/sampler_12p5" 40 12500000 > "$OUT/sampler_12p5.txt" 2>&1 || { echo SAMPLER_FAIL; tail -5 "$OUT/sampler_12p5.txt"; exit 1; }
head -40 "$OUT/sampler_12p5.txt" | cut -c1-150
echo ALL_OK
