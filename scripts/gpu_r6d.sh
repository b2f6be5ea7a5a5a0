#!/bin/bash
# r6: conv tile configurations on the layer-3/4 shapes (small M, deep K): 128x128 (auto, cfg 14),
# 256x128 (cfg 1 four-wave-column / cfg 18 sixteen-wave), 128x128 4-wave (cfg 5), 64x128 (cfg 9).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r6d"; mkdir -p "$O"
cd "$R"
WCFGS=-1 timeout -k 10 600 python -u bench/conv_igemm_probe.py --cfgs=-1,1,5,9,14,18 \
  --shapes l3.c2,l4.c2,l3.c1,l3.c3,l4.c1,l4.c3,l3.c2s2,l4.c2s2,l2.c2,l3.c1a,l4.c1a > "$O/probe.md" 2> "$O/probe.err" || { tail -20 "$O/probe.err"; exit 1; }
cat "$O/probe.md" | tail -30
