#!/bin/bash
# r03b: GPU suite, index-kernel A/B (vector histogram, nontemporal rank puts),
# HBM traffic of the C3 step (two PMC passes), library kernels (HIP events +
# rocprofv3 kernel stats).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r03b}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { echo PYTEST_FAIL; tail -40 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
i=0
for v in "1 1" "0 1" "1 0" "1 1"; do
  set -- $v
  (export BWTMI_HIST_VEC=$1 BWTMI_PUT_NT=$2; timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-fm --no-cli > "$OUT/ab_${i}_hist$1_nt$2.json" 2> "$OUT/ab_$i.err") || { echo AB_FAIL; tail -5 "$OUT/ab_$i.err"; exit 1; }
  i=$((i+1))
done
echo AB_OK
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o pmc -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-fm --no-cli > "$OUT/fetch.json" 2> "$OUT/fetch.err" || { echo FETCH_FAIL; tail -5 "$OUT/fetch.err"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o pmc -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-fm --no-cli > "$OUT/write.json" 2> "$OUT/write.err" || { echo WRITE_FAIL; tail -5 "$OUT/write.err"; exit 1; }
python3 tools/pmc_traffic.py "$OUT/fetch" "$OUT/write" "$OUT/pmc_traffic.json" && echo PMC_OK
rm -rf "$OUT/fetch" "$OUT/write"
timeout -k 10 300 python -u tools/lib_kernels.py "$OUT/lib_kernels.json" 999000 1e7 > "$OUT/lib_kernels.log" 2>&1 || { echo LIB_FAIL; tail -20 "$OUT/lib_kernels.log"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/libprof" -o lib -- python3 tools/lib_kernels.py "$OUT/lib_kernels_prof.json" 999000 1e7 > "$OUT/libprof.log" 2>&1 || { echo LIBPROF_FAIL; tail -20 "$OUT/libprof.log"; exit 1; }
find "$OUT/libprof" -name "*kernel_stats.csv" -exec cp {} "$OUT/lib_kernel_stats.csv" \;
rm -rf "$OUT/libprof"
echo ALL_OK
