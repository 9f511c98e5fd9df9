#!/bin/bash
# 2-rank rehearsal of the multi-GPU bench on a 1-GPU box: gloo collectives, both ranks on device 0
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-rehearse2}
mkdir -p "$OUT"
export TMPDIR=/tmp BWTMI_BENCH_GLOO=1
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline --no-fm --contig-bp 20000000 > "$OUT/bench2.json" 2> "$OUT/bench2.err" || { echo REHEARSE_FAIL; tail -20 "$OUT/bench2.err"; exit 1; }
cat "$OUT/bench2.json"
