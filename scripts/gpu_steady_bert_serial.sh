#!/bin/bash
# BERT-large steady-state kernel profile with the weight-gradient side stream OFF, so kernel
# durations are not stretched by concurrent execution (per-kernel costs, not overlap).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/steady"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
export CLOUDTIK_AMD_WGRAD_STREAM=0
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/bert_serial" -o bert_serial -- python3 -u "$R/bench.py" --steps 8 --warmup 4 > "$OUT/bert_serial.log" 2>&1 || exit $?
tr=$(find "$OUT/bert_serial" -name "*kernel_trace.csv" | head -1)
python3 "$R/scripts/steady_profile.py" "$tr" --delim lamb_stage1 --steps 5 --top 40 --title "bert_large (wgrad side stream off)" > "$OUT/bert_serial.md" || exit $?
rm -rf "$OUT/bert_serial"
head -3 "$OUT/bert_serial.md"
