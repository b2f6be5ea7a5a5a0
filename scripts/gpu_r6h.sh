#!/bin/bash
# r6: conv rule 3 (256x128 16-wave tiles for M <= 65536) -- conv GPU tests under it, then a
# same-box ResNet-50 A/B against rule 2.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r6h"; mkdir -p "$O"
cd "$R"
CLOUDTIK_AMD_CONV_RULE=3 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_conv_igemm.py tests/test_resnet_train_entry.py > "$O/tests.txt" 2>&1
rc=$?; tail -2 "$O/tests.txt"; [ $rc -eq 0 ] || exit $rc
bash "$R/scripts/gpu_ab_env.sh" r6h_ab CLOUDTIK_AMD_CONV_RULE "2 3" 3 resnet50
