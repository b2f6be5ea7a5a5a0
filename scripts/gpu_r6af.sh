#!/bin/bash
# Steady-state kernel traces of both bench halves on the final tree (no round check).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/r6af_prof"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for m in bert-large resnet50; do
  d=$([ $m = resnet50 ] && echo sgd_kernel || echo lamb_stage1)
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/raw_$m" -o "$m" -- python3 -u "$R/bench.py" \
    --model $m --steps 8 --warmup 4 --baseline-steps 0 > "$OUT/$m.log" 2>&1 || { tail -5 "$OUT/$m.log"; exit 1; }
  tr=$(find "$OUT/raw_$m" -name "*kernel_trace.csv" | head -1)
  python3 "$R/scripts/steady_profile.py" "$tr" --delim $d --steps 5 --top 45 --gaps 20 --title "${m}_r6_final_tree" \
    > "$OUT/steady_$m.md" || exit 1
  rm -rf "$OUT/raw_$m"
  head -3 "$OUT/steady_$m.md"
done
