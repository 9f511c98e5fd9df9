#!/bin/bash
# rocprofv3 kernel stats + the two PMC passes of the C3 step (bench.py, 1 step)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r03i}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-fm --no-cli > "$OUT/prof_bench.json" 2> "$OUT/prof.err" || { echo PROF_FAIL; tail -5 "$OUT/prof.err"; exit 1; }
find "$OUT/prof" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats_C3.csv" \;
rm -rf "$OUT/prof"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o pmc -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-fm --no-cli > "$OUT/fetch.json" 2> "$OUT/fetch.err" || { echo FETCH_FAIL; tail -5 "$OUT/fetch.err"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o pmc -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-fm --no-cli > "$OUT/write.json" 2> "$OUT/write.err" || { echo WRITE_FAIL; tail -5 "$OUT/write.err"; exit 1; }
python3 tools/pmc_traffic.py "$OUT/fetch" "$OUT/write" "$OUT/pmc_traffic.json" && echo PMC_OK
rm -rf "$OUT/fetch" "$OUT/write"
echo ALL_OK
