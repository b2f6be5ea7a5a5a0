#!/bin/bash
# GPU test suite + optional extra python commands, each under its own time limit.
# Usage: scripts/gpu_tests.sh TAG [python-args ...]   (one extra command per argument)
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=$1; shift
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/gpu_tests.txt" 2>&1 || { grep -E "FAIL|Error" "$OUT/gpu_tests.txt" | head -20; tail -40 "$OUT/gpu_tests.txt"; exit 1; }
tail -1 "$OUT/gpu_tests.txt"
i=0
for cmd in "$@"; do
  i=$((i+1))
  timeout -k 10 600 python -u $cmd > "$OUT/extra_$i.log" 2>&1 || { echo "FAILED: $cmd"; tail -30 "$OUT/extra_$i.log"; exit 1; }
  echo "== $cmd"; tail -2 "$OUT/extra_$i.log" | cut -c1-1500
done
echo ALLDONE
