#!/bin/bash
# DLRM: weight-gradient side stream on vs off, 600 timed steps, 3 interleaved rounds.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r6ap"; mkdir -p "$O"
cd "$R"
for r in 1 2 3; do
  for v in 1 0; do
    env CLOUDTIK_AMD_WGRAD_STREAM=$v timeout -k 10 200 python -u examples/ai/dlrm_synthetic.py --steps 600 --warmup 20 > "$O/d.log" 2>&1 || { tail -5 "$O/d.log"; exit 1; }
    echo "side=$v dlrm $(grep '^{' "$O/d.log" | tail -1 | grep -o '"ms_per_step": [0-9.]*')"
  done
done
