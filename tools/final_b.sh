# round-end measurement set, part B: W=8 shards (all ranks), kernel stats, PMC traffic, CLI marker trace
set -o pipefail
mkdir -p gpurun_out/r05fb
timeout -k 10 120 python3 tools/genfa.py /tmp/c3.fa C3 > /dev/null || { echo GENFA_FAIL; exit 1; }
bash tools/gpu_run.sh r05fb "py shard tools/c4_shard.py gpurun_out/r05fb/c4_shards_w8.json 16" "prof C3 --steps 5 --warmup 1" \
  "pmc C3" "mtrace C3 /tmp/c3.fa --jobs 1 --progress" "bench C3cpu --gpus 1 --steps 20 --warmup 5"
