#!/bin/bash
# One parameterised GPU-box runner (replaces the per-run tools/gpu_r03*.sh scripts).
#
# usage: tools/gpu_run.sh TAG STEP [STEP ...]      (outputs under gpurun_out/TAG/)
# each STEP is one quoted string "KIND NAME [ARGS...]" (whitespace-separated, or '|'-separated
# when an argument holds spaces: "pytest|NAME|-k|a or b"):
#   "pytest NAME [pytest args]"     GPU parity suite (-m gpu) -> NAME.log
#   "smoke NAME"                    __graft_entry__.smoke()
#   "bench NAME [bench.py args]"    one bench line -> NAME.json (+ NAME.err)
#   "prof NAME [bench.py args]"     rocprofv3 --kernel-trace --stats of a bench run -> kernel_stats_NAME.csv
#   "pmc NAME [bench.py args]"      FETCH_SIZE and WRITE_SIZE passes (one counter block per run) -> pmc_traffic_NAME.json
#   "mtrace NAME FASTA [args]"      rocprofv3 --marker-trace --kernel-trace of the CLI (+ --profile JSON)
#   "py NAME script [args]"         any python tool (tools/c4_shard.py, tools/lib_kernels.py, ...) -> NAME.log
# Every step runs under its own time limit; the first failing step ends the call.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
summ() {   # one-line digest of a bench JSON line
  python3 - "$1" <<'EOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
g = d.get("golden") or {}
r = d.get("roofline") or {}
print(d["config"]["workload"].split(":")[0], d["n_gpus"], d["value"], d["ms_per_step"], "golden", g.get("match"),
      "calls", d["calls_ms_per_step"], "roof", r.get("kernel"), r.get("frac"), "stages", d["stage_ms_last_step"])
print("kernels", list(d["kernels_ms_per_step"].items())[:14])
EOF
}
for step in "$@"; do
  if [[ $step == *"|"* ]]; then   # fields separated by '|' may hold spaces: "pytest|x|-k|a or b"
    IFS='|' read -r -a A <<< "$step"
  else
    read -r -a A <<< "$step"
  fi
  kind=${A[0]}; name=${A[1]}; args=("${A[@]:2}")
  echo "== $kind $name ${args[*]}"
  case $kind in
    pytest)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${args[@]}" \
        > "$OUT/$name.log" 2>&1 || { echo PYTEST_FAIL; tail -40 "$OUT/$name.log"; exit 1; }
      tail -1 "$OUT/$name.log" ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/$name.log" 2>&1 \
        || { echo SMOKE_FAIL; tail -20 "$OUT/$name.log"; exit 1; }
      tail -1 "$OUT/$name.log" ;;
    bench)
      timeout -k 10 600 python bench.py "${args[@]}" > "$OUT/$name.json" 2> "$OUT/$name.err" \
        || { echo BENCH_FAIL; tail -20 "$OUT/$name.err"; exit 1; }
      summ "$OUT/$name.json" ;;
    prof)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$name" -o run -- \
        python3 bench.py --no-cpu-baseline --no-fm --no-cli "${args[@]}" > "$OUT/prof_$name.json" 2> "$OUT/prof_$name.err" \
        || { echo PROF_FAIL; tail -5 "$OUT/prof_$name.err"; exit 1; }
      find "$OUT/prof_$name" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats_$name.csv" \;
      rm -rf "$OUT/prof_$name"
      head -16 "$OUT/kernel_stats_$name.csv" | cut -d, -f1-6 ;;
    pmc)
      for ctr in FETCH_SIZE WRITE_SIZE; do
        timeout -k 10 -s KILL 300 rocprofv3 --pmc $ctr --output-format csv -d "$OUT/pmc_${name}_$ctr" -o pmc -- \
          python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-fm --no-cli "${args[@]}" \
          > "$OUT/pmc_${name}_$ctr.json" 2> "$OUT/pmc_${name}_$ctr.err" \
          || { echo PMC_FAIL $ctr; tail -5 "$OUT/pmc_${name}_$ctr.err"; exit 1; }
      done
      python3 tools/pmc_traffic.py "$OUT/pmc_${name}_FETCH_SIZE" "$OUT/pmc_${name}_WRITE_SIZE" "$OUT/pmc_traffic_$name.json" \
        || { echo PMC_PARSE_FAIL; exit 1; }
      rm -rf "$OUT/pmc_${name}_FETCH_SIZE" "$OUT/pmc_${name}_WRITE_SIZE" ;;
    sq)   # one SQ counter pass over the kernels matching a regex ('+' stands for '|'): "sq NAME CTR,CTR,... REGEX [bench.py args]"
      IFS=',' read -r -a CTRS <<< "${args[0]}"
      RX=${args[1]//+/|}
      timeout -k 10 -s KILL 180 rocprofv3 --pmc "${CTRS[@]}" --kernel-include-regex "$RX" --output-format csv \
        -d "$OUT/sq_$name" -o sq -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-fm --no-cli "${args[@]:2}" \
        > "$OUT/sq_$name.json" 2> "$OUT/sq_$name.err" || { echo SQ_FAIL; tail -5 "$OUT/sq_$name.err"; exit 1; }
      python3 tools/pmc_sq.py "$OUT/sq_$name" > "$OUT/sq_$name.txt" && cat "$OUT/sq_$name.txt"
      rm -rf "$OUT/sq_$name" ;;
    mtrace)   # roctx stage ranges + kernels of one CLI run: "mtrace NAME FASTA [bwt.py args]"
      timeout -k 10 600 rocprofv3 --marker-trace --kernel-trace --output-format csv -d "$OUT/mt_$name" -o run -- \
        python3 bwt-algorithm_amd/bwt.py "${args[@]}" -o "$OUT/mt_$name.tab" --profile "$OUT/profile_$name.json" \
        > "$OUT/mt_$name.log" 2>&1 || { echo MTRACE_FAIL; tail -5 "$OUT/mt_$name.log"; exit 1; }
      find "$OUT/mt_$name" -name "*marker_api_trace.csv" -exec cp {} "$OUT/marker_trace_$name.csv" \;
      find "$OUT/mt_$name" -name "*kernel_trace.csv" -exec cp {} "$OUT/kernel_trace_$name.csv" \;
      rm -rf "$OUT/mt_$name" "$OUT/mt_$name.tab"
      python3 tools/stage_ranges.py "$OUT/marker_trace_$name.csv" "$OUT/kernel_trace_$name.csv" > "$OUT/stage_ranges_$name.txt" \
        && cat "$OUT/stage_ranges_$name.txt" ;;
    py)
      timeout -k 10 600 python -u "${args[@]}" > "$OUT/$name.log" 2>&1 || { echo PY_FAIL; tail -30 "$OUT/$name.log"; exit 1; }
      tail -15 "$OUT/$name.log" ;;
    *)
      echo "unknown step kind: $kind"; exit 2 ;;
  esac
done
echo ALL_OK
