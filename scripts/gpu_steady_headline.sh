#!/bin/bash
# Steady-state kernel profiles of the two headline benches (default settings: gradient side
# stream on, so per-kernel times include overlap).  Traces are summarised on the box.
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
  python3 "$R/scripts/steady_profile.py" "$tr" --delim "$delim" --steps 5 --top 40 --title "$name" > "$OUT/$name.md" || return $?
  rm -rf "$OUT/$name"
  head -3 "$OUT/$name.md"
}
prof bert_large lamb_stage1 -- python3 -u "$R/bench.py" --model bert-large --steps 8 --warmup 4 \
 && prof resnet50 sgd_kernel -- python3 -u "$R/bench.py" --model resnet50 --steps 8 --warmup 4
