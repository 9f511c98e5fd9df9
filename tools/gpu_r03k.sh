#!/bin/bash
# r03k: device recompute CLI goldens; host sampler of the C3 step with the
# fold's recomputes on the host / on the device; k_recompute kernel time
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r03k}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_recompute.py -x -v --timeout 500 --timeout-method thread > "$OUT/pytest_rc.log" 2>&1 || { echo RC_FAIL; tail -40 "$OUT/pytest_rc.log"; exit 1; }
tail -1 "$OUT/pytest_rc.log"
for pd in 0 1; do
  (export BWTMI_POST_DEVICE=$pd; timeout -k 10 300 python -u tools/sampler.py "$OUT/samp_pd$pd" 10 > "$OUT/samp_pd$pd.log" 2>&1) || { echo SAMP_FAIL $pd; tail -20 "$OUT/samp_pd$pd.log"; exit 1; }
  rm -f "$OUT/samp_pd$pd.raw" "$OUT/samp_pd$pd.raw.chains"
done
echo SAMP_OK
BWTMI_POST_DEVICE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-fm --no-cli > "$OUT/prof_bench.json" 2> "$OUT/prof.err" || { echo PROF_FAIL; tail -5 "$OUT/prof.err"; exit 1; }
find "$OUT/prof" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats_pd1.csv" \;
rm -rf "$OUT/prof"
echo ALL_OK
