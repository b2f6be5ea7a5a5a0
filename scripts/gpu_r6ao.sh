#!/bin/bash
# Weight-gradient side stream as the process default (models that do not choose): on vs off
# for the models that do not set it themselves -- DLRM, T5 and RNN-T training, Mask R-CNN step.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r6ao"; mkdir -p "$O"
cd "$R"
for r in 1 2; do
  for v in 1 0; do
    env CLOUDTIK_AMD_WGRAD_STREAM=$v timeout -k 10 200 python -u examples/ai/dlrm_synthetic.py --steps 60 > "$O/d.log" 2>&1 || { tail -5 "$O/d.log"; exit 1; }
    echo "side=$v dlrm $(grep '^{' "$O/d.log" | tail -1 | grep -o '"ms_per_step": [0-9.]*')"
    env CLOUDTIK_AMD_WGRAD_STREAM=$v timeout -k 10 300 python -u examples/ai/inference_benchmark.py --models rnnt,t5_base --train > "$O/t.log" 2>&1 || { tail -5 "$O/t.log"; exit 1; }
    echo "side=$v $(grep '^{' "$O/t.log" | grep -o '"model": "[a-z0-9_]*"\|"ms_per_batch": [0-9.]*' | tr '\n' ' ')"
    env CLOUDTIK_AMD_WGRAD_STREAM=$v timeout -k 10 300 python -u bench/maskrcnn_step.py > "$O/m.log" 2>&1 || { tail -5 "$O/m.log"; exit 1; }
    echo "side=$v maskrcnn $(grep "flat-opt step" "$O/m.log" | tail -3 | tr "\n" " ")"
  done
done
