#!/bin/bash
# LayerNorm kernels with and without the regenerated dropout mask (p 0.1 vs 0), interleaved.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
for r in 1 2; do
  for p in 0.1 0.0; do
    timeout -k 10 120 python3 bench/ln_from_y_probe.py --rounds 3 --p $p 2>/dev/null | tail -1 | sed "s/^/p=$p: /" || exit 1
  done
done
