# round-end measurement set, part A: GPU suite, smoke, bench lines
set -o pipefail
bash tools/gpu_run.sh r05ia "pytest full" "smoke smoke" "bench C3 --gpus 1 --steps 20 --warmup 5" \
  "bench C4 --workload C4 --steps 10 --warmup 3 --no-cpu-baseline --no-fm --no-cli" \
  "bench C5 --workload C5 --steps 10 --warmup 3 --no-cpu-baseline --no-fm --no-cli" \
  "bench C3N --workload C3N --steps 10 --warmup 3 --no-cpu-baseline --no-fm --no-cli"
