#!/bin/bash
# Kernel + HIP API trace of the ResNet-50 bench half; attributes main-stream idle gaps to a late
# host launch or to a GPU-side hold (scripts/launch_lag.py).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/launch_lag"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
name=${1:-rn}; shift
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --output-format csv -d "$OUT/$name" -o "$name" -- python3 -u "$R/bench.py" --model resnet50 --steps 8 --warmup 4 "$@" > "$OUT/$name.log" 2>&1 || { tail -5 "$OUT/$name.log"; exit 1; }
kt=$(find "$OUT/$name" -name "*kernel_trace.csv" | head -1)
at=$(find "$OUT/$name" -name "*hip_api_trace.csv" | head -1)
python3 "$R/scripts/launch_lag.py" "$kt" "$at" --delim sgd_kernel > "$OUT/$name.md" || exit 1
rm -rf "$OUT/$name"
cat "$OUT/$name.md"
