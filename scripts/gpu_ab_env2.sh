#!/bin/bash
# A/B an env switch on one bench model: VAR, VALS, MODEL, ROUNDS
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/ab_env2"; mkdir -p "$OUT"
for r in $(seq 1 ${ROUNDS:-1}); do
  for v in $VALS; do
    env "$VAR=$v" timeout -k 10 300 python3 "$R/bench.py" --model ${MODEL:-bert-large} --steps 20 --warmup 5 > "$OUT/${VAR}_${v}_$r.log" 2>&1 || { echo "run $v failed"; tail -5 "$OUT/${VAR}_${v}_$r.log"; exit 1; }
    echo "$VAR=$v round $r: $(grep -o '"ms_per_step": [0-9.]*' "$OUT/${VAR}_${v}_$r.log" | head -1)"
  done
done
