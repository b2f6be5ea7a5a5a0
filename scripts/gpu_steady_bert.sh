#!/bin/bash
# Steady-state kernel profile of the BERT-large bench half (HEAD routing).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/steady_bert"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
name=${1:-bert}
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/$name" -o "$name" -- python3 -u "$R/bench.py" --model bert-large --steps 8 --warmup 4 > "$OUT/$name.log" 2>&1 || { tail -5 "$OUT/$name.log"; exit 1; }
tr=$(find "$OUT/$name" -name "*kernel_trace.csv" | head -1)
python3 "$R/scripts/steady_profile.py" "$tr" --delim lamb_stage1 --steps 5 --title "$name" > "$OUT/$name.md" || exit 1
rm -rf "$OUT/$name"
head -40 "$OUT/$name.md"
