#!/bin/bash
# BERT-large steady-state kernel profile, default configuration (WS=0: side stream off)
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/steady"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
name=bert_large${TAG:-}
CLOUDTIK_AMD_WGRAD_STREAM=${WS:-1} timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/$name" -o $name -- python3 -u "$R/bench.py" --model bert-large --steps 8 --warmup 4 > "$OUT/$name.log" 2>&1 || exit $?
tr=$(find "$OUT/$name" -name "*kernel_trace.csv" | head -1)
python3 "$R/scripts/steady_profile.py" "$tr" --delim lamb_stage1 --steps 5 --top 40 --title "$name" > "$OUT/$name.md" || exit $?
rm -rf "$OUT/$name"
head -30 "$OUT/$name.md"
