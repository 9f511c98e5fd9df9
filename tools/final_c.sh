# same-box 1-GPU C4 line and W=8 shards (the 8-rank projection's ratio), and the CLI marker trace
set -o pipefail
mkdir -p gpurun_out/r05ic
timeout -k 10 120 python3 tools/genfa.py /tmp/c3.fa C3 > /dev/null || { echo GENFA_FAIL; exit 1; }
bash tools/gpu_run.sh r05ic "bench C4 --workload C4 --steps 10 --warmup 3 --no-cpu-baseline --no-fm --no-cli" \
  "py shard tools/c4_shard.py gpurun_out/r05ic/c4_shards_w8.json 16" \
  "bench C4b --workload C4 --steps 10 --warmup 3 --no-cpu-baseline --no-fm --no-cli" \
  "mtrace C3 /tmp/c3.fa --jobs 1 --progress"
