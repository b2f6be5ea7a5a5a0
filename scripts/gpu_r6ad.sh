#!/bin/bash
# ResNet-50 knob re-check on the final tree (one knob changed per run, 2 interleaved rounds).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/r6ad"; mkdir -p "$OUT"
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 240 python3 "$R/bench.py" --model resnet50 --steps 30 --warmup 5 --baseline-steps 0 \
    > "$OUT/$tag.log" 2>&1 || { echo "$tag failed"; tail -5 "$OUT/$tag.log"; exit 1; }
  echo "$tag: $(grep -o '"resnet50_ms_per_step": [0-9.]*' "$OUT/$tag.log" | head -1)"
}
for r in 1 2; do
  run default_$r CLOUDTIK_AMD_NOOP=1 || exit 1
  run down_stream_$r CLOUDTIK_AMD_RESNET_DOWN_STREAM=1 || exit 1
  run phase_streams_$r CLOUDTIK_AMD_CONV_PHASE_STREAMS=1 || exit 1
  run bn_ew2_$r CLOUDTIK_AMD_BN_EW=2 || exit 1
  run phase_batch_$r CLOUDTIK_AMD_CONV_PHASE_BATCH=1 || exit 1
done
