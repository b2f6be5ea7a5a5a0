#!/bin/bash
# Steady-state kernel profiles (per-step busy time vs step span) of the headline benches and
# Mask R-CNN training.  Traces are summarised on the box and deleted (they are large).
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
  python3 "$R/scripts/steady_profile.py" "$tr" --delim "$delim" --steps 5 --title "$name" > "$OUT/$name.md" || return $?
  rm -rf "$OUT/$name"
  head -3 "$OUT/$name.md"
}
prof maskrcnn_train sgd_kernel -- python3 -u "$R/examples/ai/inference_benchmark.py" --train --models maskrcnn --steps 8 --warmup 4 \
 && prof bert_large lamb_stage1 -- python3 -u "$R/bench.py" --steps 8 --warmup 4 \
 && prof resnet50 sgd_kernel -- python3 -u "$R/bench.py" --model resnet50 --steps 8 --warmup 4
