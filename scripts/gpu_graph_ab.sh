#!/bin/bash
# whole-step hipGraph: GPU tests, then ResNet-50 bench with --graph off / on (two rounds)
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/graph_ab"; mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_graph_step_gpu.py > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
tail -2 "$OUT/tests.log"
for r in 1 2; do
  for g in off on; do
    timeout -k 10 300 python3 "$R/bench.py" --model resnet50 --steps 20 --warmup 5 --graph $g > "$OUT/rn_${g}_$r.log" 2>&1 || { echo "run $g/$r failed"; tail -8 "$OUT/rn_${g}_$r.log"; exit 1; }
    echo "graph=$g round $r: $(grep -o '"ms_per_step": [0-9.]*' "$OUT/rn_${g}_$r.log") $(grep -o '"loss_last_step": [0-9.]*' "$OUT/rn_${g}_$r.log") $(grep -o '"hip_graph": [a-z]*' "$OUT/rn_${g}_$r.log")"
  done
done
