#!/bin/bash
# A/B several env configurations of one bench model, interleaved over rounds:
#   scripts/gpu_ab_multi.sh TAG ROUNDS MODEL "A=1,B=2" "A=0" ...   ("-" = defaults)
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=$1; ROUNDS=$2; MODEL=$3; shift 3
OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
for r in $(seq 1 "$ROUNDS"); do
  i=0
  for cfg in "$@"; do
    i=$((i + 1))
    envs=()
    [ "$cfg" != "-" ] && IFS=',' read -r -a envs <<< "$cfg"
    log="$OUT/cfg${i}_$r.log"
    env "${envs[@]}" timeout -k 10 300 python3 "$R/bench.py" --model "$MODEL" --steps 20 --warmup 5 > "$log" 2>&1 \
      || { echo "config '$cfg' round $r failed"; tail -5 "$log"; exit 1; }
    echo "[$cfg] round $r: $(grep -o '"ms_per_step": [0-9.]*' "$log")"
  done
done
