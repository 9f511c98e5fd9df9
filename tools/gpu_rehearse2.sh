#!/bin/bash
# 2-rank rehearsal of the multi-GPU bench on a one-GPU box: both ranks on device 0,
# host transport for the collectives (BWTMI_BENCH_GLOO=1); the C4 shared-FASTA path.
# usage: tools/gpu_rehearse2.sh TAG [bench args]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-rehearse}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp BWTMI_BENCH_GLOO=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29611 WORLD_SIZE=2 LOCAL_WORLD_SIZE=2
pids=()
for R in 0 1; do
  RANK=$R LOCAL_RANK=$R timeout -k 10 600 python bench.py --gpus 2 --no-cpu-baseline --no-fm "$@" > "$OUT/r$R.json" 2> "$OUT/r$R.err" &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=$?; done
cat "$OUT/r0.json"
[ $rc -eq 0 ] && echo REHEARSE_OK || { echo REHEARSE_FAIL $rc; tail -5 "$OUT/r0.err" "$OUT/r1.err"; exit 1; }
