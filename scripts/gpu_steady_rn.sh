#!/bin/bash
# Steady-state kernel profile of the ResNet-50 half of the bench (HEAD routing).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/steady_rn"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
name=${1:-resnet50}
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/$name" -o "$name" -- python3 -u "$R/bench.py" --model resnet50 --steps 8 --warmup 4 > "$OUT/$name.log" 2>&1 || { tail -5 "$OUT/$name.log"; exit 1; }
tr=$(find "$OUT/$name" -name "*kernel_trace.csv" | head -1)
python3 "$R/scripts/steady_profile.py" "$tr" --delim sgd_kernel --steps 5 --gaps 20 --title "$name" > "$OUT/$name.md" || exit 1
rm -rf "$OUT/$name"
head -3 "$OUT/$name.md"
