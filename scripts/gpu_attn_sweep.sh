#!/bin/bash
# Attention forward occupancy sweep (waves per SIMD) + BERT-large bench per setting.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/attn_sweep"
mkdir -p "$OUT"
cd "$R"
for w in 1 2 3; do
  CLOUDTIK_AMD_ATTN_FWD_WPE=$w timeout -k 10 120 python bench/attention_bench.py > "$OUT/attn_w$w.json" 2>&1 || { tail -5 "$OUT/attn_w$w.json"; exit 1; }
  echo "wpe $w: $(tail -1 "$OUT/attn_w$w.json" | cut -c1-400)"
done
for w in 2 3; do
  CLOUDTIK_AMD_ATTN_FWD_WPE=$w timeout -k 10 300 python bench.py --model bert-large --steps 20 --warmup 5 > "$OUT/bert_w$w.log" 2>&1 || { tail -5 "$OUT/bert_w$w.log"; exit 1; }
  echo "bert wpe $w: $(tail -1 "$OUT/bert_w$w.log" | cut -c1-200)"
done
