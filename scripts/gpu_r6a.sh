#!/bin/bash
# r6 first call: round check (bench, GPU tests, smoke) then a ResNet-50 kernel trace kept whole
# for gap analysis (which stream / event a main-stream gap waits on).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
bash "$R/scripts/gpu_round_check.sh" r6a || exit $?
OUT="$R/gpurun_out/r6a_rn"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/raw" -o rn -- python3 -u "$R/bench.py" --model resnet50 --steps 8 --warmup 4 > "$OUT/rn.log" 2>&1 || { tail -5 "$OUT/rn.log"; exit 1; }
tr=$(find "$OUT/raw" -name "*kernel_trace.csv" | head -1)
cp "$tr" "$OUT/rn_kernel_trace.csv"
rm -rf "$OUT/raw"
python3 "$R/scripts/steady_profile.py" "$OUT/rn_kernel_trace.csv" --delim sgd_kernel --steps 5 --gaps 20 --title rn_r6a > "$OUT/rn.md" && head -3 "$OUT/rn.md"
