#!/bin/bash
# SSD-ResNet34 training (1,099 vs 1,247 images/s in round 2): which routing moved it.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r6as"; mkdir -p "$O"
cd "$R"
for r in 1 2; do
  for v in "CLOUDTIK_AMD_NOOP=1" "CLOUDTIK_AMD_WGRAD_STREAM=0" "CLOUDTIK_AMD_CONV_IGEMM=0" "CLOUDTIK_AMD_DEFER_WGRAD=0"; do
    env $v timeout -k 10 300 python -u examples/ai/inference_benchmark.py --models ssd_resnet34_300 --train > "$O/s.log" 2>&1 || { echo "$v failed"; tail -5 "$O/s.log"; exit 1; }
    echo "$v: $(grep '^{' "$O/s.log" | tail -1 | grep -o '"ms_per_batch": [0-9.]*')"
  done
done
