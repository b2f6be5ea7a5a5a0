#!/bin/bash
# DLRM with its MLP weight gradients in line (models/dlrm.py): GPU tests, then 3 runs.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r6aq"; mkdir -p "$O"
cd "$R"
timeout -k 10 300 python -u -m pytest tests -m gpu -k "dlrm or embedding or interaction" -x -q --timeout 120 --timeout-method thread > "$O/tests.txt" 2>&1 || { tail -20 "$O/tests.txt"; exit 1; }
tail -1 "$O/tests.txt"
for r in 1 2 3; do
  timeout -k 10 200 python -u examples/ai/dlrm_synthetic.py --steps 600 --warmup 20 > "$O/d.log" 2>&1 || { tail -5 "$O/d.log"; exit 1; }
  grep '^{' "$O/d.log" | tail -1
done
