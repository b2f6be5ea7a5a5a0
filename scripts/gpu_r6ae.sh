#!/bin/bash
# BERT-large knob re-check on the final tree (one knob changed per run, 2 interleaved rounds).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/r6ae"; mkdir -p "$OUT"
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 240 python3 "$R/bench.py" --model bert-large --steps 20 --warmup 5 --baseline-steps 0 \
    > "$OUT/$tag.log" 2>&1 || { echo "$tag failed"; tail -5 "$OUT/$tag.log"; exit 1; }
  echo "$tag: $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$tag.log" | head -1)"
}
for r in 1 2; do
  run default_$r CLOUDTIK_AMD_NOOP=1 || exit 1
  run group_m2_$r CLOUDTIK_AMD_GEMM_GROUP_M=2 || exit 1
  run group_m8_$r CLOUDTIK_AMD_GEMM_GROUP_M=8 || exit 1
  run stagger_auto_$r CLOUDTIK_AMD_GEMM_STAGGER=-1 || exit 1
  run attn_wpe2_$r CLOUDTIK_AMD_ATTN_FWD_WPE=2 || exit 1
  run attn_persist0_$r CLOUDTIK_AMD_ATTN_PERSIST=0 || exit 1
done
