#!/bin/bash
# A/B of BERT-large bench settings on one box: attention fwd occupancy x TunableOp table path.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/ab"; mkdir -p "$OUT"; cd "$R"
for cfg in "1 1" "1 0" "2 1" "2 0" "1 1"; do
  set -- $cfg
  CLOUDTIK_AMD_ATTN_FWD_WPE=$1 CLOUDTIK_BENCH_TUNE_DIRECT=$2 timeout -k 10 300 python bench.py --model bert-large --steps 20 --warmup 5 > "$OUT/b_$1_$2.log" 2>&1 || { tail -5 "$OUT/b_$1_$2.log"; exit 1; }
  echo "wpe=$1 direct=$2: $(grep TunableOp "$OUT/b_$1_$2.log" | cut -c1-120) $(tail -1 "$OUT/b_$1_$2.log" | cut -c100-170)"
done
