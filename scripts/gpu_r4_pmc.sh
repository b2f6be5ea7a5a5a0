#!/bin/bash
# Round 4: the north-star control-plane slice on the GPU, then counter tables of both models.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r4pmc"
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python -u -m pytest tests/test_northstar_gpu.py -m gpu -x -v --timeout 500 --timeout-method thread > "$O/northstar.txt" 2>&1
rc=$?
tail -3 "$O/northstar.txt"
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" "$O/northstar.txt" | head -20; exit $rc; }
bash scripts/gpu_pmc.sh r4pmc bert-large "gemm_nt|Cijk|attn_|ln_|lamb|xent|bias_act|splitk" && \
bash scripts/gpu_pmc.sh r4pmc resnet50 "conv_|bn_|sgd|splitk|maxpool"
