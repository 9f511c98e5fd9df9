#!/bin/bash
# A/B over environment settings on the C3 bench: each argument after TAG is one
# variant, a comma-separated list of VAR=VALUE (or "base"); prints the stage and
# kernel times of each
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-env_ab}; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for v in "$@"; do
  i=$((i+1))
  envs=""; [ "$v" != base ] && envs=$(echo "$v" | tr ',' ' ')
  env $envs timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-fm ${BENCH_ARGS:-} > "$OUT/v$i.json" 2> "$OUT/v$i.err" || { echo FAIL "$v"; tail -5 "$OUT/v$i.err"; exit 1; }
  python - "$OUT/v$i.json" "$v" <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k=d["kernels_ms_per_step"]
sel={n:k[n] for n in ("radix_scatter_kv8","radix_partition_kv8","radix_hist","dna_rank0","dna_heads","dna_rank_put","dna_ls_keys") if n in k}
print(sys.argv[2],"value",round(d["value"],1),"index",d["stage_ms_last_step"]["index"],"roof",round(d["roofline"]["frac"],3),d["roofline"].get("kernel"),sel,"sha",d["golden"]["match"])
PY
done
