#!/bin/bash
# BERT-large: the QKV forward (hipBLASLt stream-K, ~1.0 PF/s in the step) on the in-tree one-tile
# or streamed kernel instead, every other site unchanged.  3 interleaved rounds.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/r6aa"; mkdir -p "$OUT"
run() {  # tag, env assignments...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python3 "$R/bench.py" --model bert-large --steps 20 --warmup 5 --baseline-steps 0 \
    > "$OUT/$tag.log" 2>&1 || { echo "$tag failed"; tail -5 "$OUT/$tag.log"; exit 1; }
  echo "$tag: $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$tag.log" | head -1) $(grep -o '"sclk_mhz": {"mean": [0-9.]*' "$OUT/$tag.log" | head -1)"
}
for r in 1 2 3; do
  run default_$r CLOUDTIK_AMD_NOOP=1 || exit 1
  run onetile_qkv_$r CLOUDTIK_AMD_ONETILE_GEMM=qkv,do,dx_attn,dx_ffn || exit 1
  run stream_qkv_$r CLOUDTIK_AMD_STREAM_GEMM=qkv || exit 1
done
