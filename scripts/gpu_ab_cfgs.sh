#!/bin/bash
# Interleaved A/B over whole env configurations on one box:
#   scripts/gpu_ab_cfgs.sh TAG ROUNDS MODEL "NAME1:VAR=v;VAR2=w" "NAME2:..." ...
# (an empty env list "base:" runs the defaults; ";" separates VAR=value pairs).  Prints ms_per_step per config per round.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=$1; ROUNDS=$2; MODEL=$3; shift 3
OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
for r in $(seq 1 "$ROUNDS"); do
  for cfg in "$@"; do
    name=${cfg%%:*}; vars=${cfg#*:}
    envs=(); IFS=";" read -ra kv <<< "$vars"; for e in "${kv[@]}"; do [ -n "$e" ] && envs+=("$e"); done
    env "${envs[@]}" timeout -k 10 300 python3 "$R/bench.py" --model "$MODEL" --steps 20 --warmup 5 \
        > "$OUT/${name}_$r.log" 2>&1 || { echo "run $name/$r failed"; tail -5 "$OUT/${name}_$r.log"; exit 1; }
    echo "$name round $r: $(grep -o '"ms_per_step": [0-9.]*' "$OUT/${name}_$r.log")"
  done
done
