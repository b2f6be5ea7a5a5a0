#!/bin/bash
# A/B one env switch on a bench model: scripts/gpu_ab_env.sh TAG VAR "val1 val2" [rounds] [model]
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=$1; VAR=$2; VALS=$3; ROUNDS=${4:-2}; MODEL=${5:-bert-large}
OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
for r in $(seq 1 $ROUNDS); do
  for v in $VALS; do
    env "$VAR=$v" timeout -k 10 300 python3 "$R/bench.py" --model $MODEL --steps 20 --warmup 5 > "$OUT/${VAR}_${v}_$r.log" 2>&1 || { echo "run $v/$r failed"; tail -5 "$OUT/${VAR}_${v}_$r.log"; exit 1; }
    echo "$VAR=$v round $r: $(grep -o '"ms_per_step": [0-9.]*' "$OUT/${VAR}_${v}_$r.log")"
  done
done
