#!/bin/bash
# ResNet-50 A/B of one environment switch, interleaved on one box: VAR=name A=value B=value
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/rnab"
mkdir -p "$O"
cd "$R"
for r in 1 2 3; do
  for v in "$A" "$B"; do
    env "$VAR=$v" timeout -k 10 240 python -u bench.py --model ${MODEL:-resnet50} --steps 20 --warmup 5 > "$O/rn_${v}_$r.json" 2> "$O/rn_${v}_$r.err" || exit $?
    echo "$VAR=$v round $r: $(grep -o '"ms_per_step": [0-9.]*' "$O/rn_${v}_$r.json")"
  done
done
