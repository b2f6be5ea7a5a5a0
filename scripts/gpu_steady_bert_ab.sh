#!/bin/bash
# Steady-state BERT-large kernel profiles with the fused FFN epilogues off / on
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/steady"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
prof() {  # name delim -- cmd...
  local name=$1 delim=$2; shift 3
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/$name" -o "$name" -- "$@" > "$OUT/$name.log" 2>&1 || return $?
  local tr
  tr=$(find "$OUT/$name" -name "*kernel_trace.csv" | head -1)
  python3 "$R/scripts/steady_profile.py" "$tr" --delim "$delim" --steps 5 --title "$name" --top 40 > "$OUT/$name.md" || return $?
  rm -rf "$OUT/$name"
  head -3 "$OUT/$name.md"
}
CLOUDTIK_AMD_WGRAD_STREAM=${WS:-1} CLOUDTIK_AMD_FUSED_FFN_FWD=0 CLOUDTIK_AMD_FUSED_FFN_DGRAD=0 prof bert_large_unfused${TAG:-} lamb_stage1 -- python3 -u "$R/bench.py" --model bert-large --steps 8 --warmup 4 \
 && CLOUDTIK_AMD_WGRAD_STREAM=${WS:-1} CLOUDTIK_AMD_FUSED_FFN_FWD=1 CLOUDTIK_AMD_FUSED_FFN_DGRAD=1 prof bert_large_fused${TAG:-} lamb_stage1 -- python3 -u "$R/bench.py" --model bert-large --steps 8 --warmup 4
