#!/bin/bash
# Detection-family training throughput on the final tree (vs profiles/detection_family.md).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r6ar"; mkdir -p "$O"
cd "$R"
timeout -k 10 600 python -u examples/ai/inference_benchmark.py --models maskrcnn,retinanet,ssd_resnet34_300 --train > "$O/train_det.log" 2>&1 || { tail -8 "$O/train_det.log"; exit 1; }
grep '^{' "$O/train_det.log" | cut -c1-220
