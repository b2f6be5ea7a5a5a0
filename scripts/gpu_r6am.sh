#!/bin/bash
# Model-family pass on the final tree: DLRM training, the reference's inference workloads
# (vision + T5 + RNN-T), and RNN-T / T5 training, each under its own time limit.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r6am"; mkdir -p "$O"
cd "$R"
timeout -k 10 240 python -u examples/ai/dlrm_synthetic.py > "$O/dlrm.log" 2>&1 || { tail -5 "$O/dlrm.log"; exit 1; }
grep '^{' "$O/dlrm.log" | tail -1
timeout -k 10 480 python -u examples/ai/inference_benchmark.py > "$O/infer_vision.log" 2>&1 || { tail -5 "$O/infer_vision.log"; exit 1; }
grep '^{' "$O/infer_vision.log" | cut -c1-220
timeout -k 10 300 python -u examples/ai/inference_benchmark.py --models t5_base,rnnt > "$O/infer_seq.log" 2>&1 || { tail -5 "$O/infer_seq.log"; exit 1; }
grep '^{' "$O/infer_seq.log" | cut -c1-220
timeout -k 10 300 python -u examples/ai/inference_benchmark.py --models rnnt,t5_base --train > "$O/train_seq.log" 2>&1 || { tail -5 "$O/train_seq.log"; exit 1; }
grep '^{' "$O/train_seq.log" | cut -c1-220
