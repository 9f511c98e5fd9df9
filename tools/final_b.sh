# round-end measurement set, part B: C3 kernel stats and PMC traffic
set -o pipefail
bash tools/gpu_run.sh r05ib "prof C3 --steps 5 --warmup 1" "pmc C3"
