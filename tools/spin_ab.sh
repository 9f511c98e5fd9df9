set -o pipefail
mkdir -p gpurun_out/r05ge
export C4_SHARD_RANKS=0,3
for sp in -1 10 -1 10; do
  BWTMI_POOL_SPIN_US=$sp timeout -k 10 300 python -u tools/c4_shard.py gpurun_out/r05ge/sh_$sp.json 16 > gpurun_out/r05ge/sh_$sp.log 2>&1 || { echo SHARD_FAIL; tail -5 gpurun_out/r05ge/sh_$sp.log; exit 1; }
  python3 -c "
import json,sys; d=json.load(open('gpurun_out/r05ge/sh_$sp.json')); print('spin $sp', [(r['rank'], r['step_ms'], r['calls_ms']['postprocess'], r['calls_ms']['write']) for r in d['runs']])"
  BWTMI_POOL_SPIN_US=$sp timeout -k 10 120 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-fm --no-cli > gpurun_out/r05ge/C3_$sp.json 2>/dev/null || { echo BENCH_FAIL; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/r05ge/C3_$sp.json').read().strip().splitlines()[-1]); print('C3 spin $sp', d['value'], d['calls_ms_per_step'], d['host_per_step'])"
done
