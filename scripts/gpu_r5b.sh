#!/bin/bash
# r5: telemetry probe, GPU test suite, then the two-model gloo run on one GPU (2 ranks share it):
# BERT (weight gradients in line) then ResNet-50 (side stream) in the same rank processes.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/${1:-r5b}"
mkdir -p "$O"
cd "$R"
timeout -k 10 120 python -u bench/telemetry_probe.py > "$O/telemetry_probe.txt" 2>&1 \
 && timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$O/gpu_tests.txt" 2>&1 \
 && tail -1 "$O/gpu_tests.txt" \
 && timeout -k 10 400 python -u bench.py --gpus 2 --dist-backend gloo --model all --steps 6 --warmup 2 --batch 64 --rn-batch 64 > "$O/gloo2.log" 2> "$O/gloo2.err" \
 && tail -c 400 "$O/gloo2.log"
rc=$?
[ $rc -eq 0 ] || { grep -E "FAIL|Error" "$O/gpu_tests.txt" 2>/dev/null | head; tail -20 "$O/gloo2.err" 2>/dev/null; }
exit $rc
