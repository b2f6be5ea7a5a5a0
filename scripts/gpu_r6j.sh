#!/bin/bash
# r6: LayerNorm backward from the block output -- numerics (kernel test, headline-routing parity
# vs fp32 HF), then a same-box BERT-large A/B of CLOUDTIK_AMD_LN_FROM_Y.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r6j"; mkdir -p "$O"
cd "$R"
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_ops_gpu.py tests/test_model_parity.py tests/test_bert_pretrain.py > "$O/tests.txt" 2>&1
rc=$?; grep -E "passed|failed|FAIL|Error" "$O/tests.txt" | tail -5; [ $rc -eq 0 ] || exit $rc
bash "$R/scripts/gpu_ab_env.sh" r6j_ab CLOUDTIK_AMD_LN_FROM_Y "0 1" 3 bert-large
