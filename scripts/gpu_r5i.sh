#!/bin/bash
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=${1:-r5i}
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python -u -m pytest tests/test_gemm_nt_gpu.py tests/test_model_parity.py -m gpu -x -v --timeout 200 --timeout-method thread > "$O/tests.txt" 2>&1 \
 && tail -1 "$O/tests.txt" \
 && timeout -k 10 120 python -u bench/epi_burst_probe.py > "$O/epi.txt" 2>&1 && tail -1 "$O/epi.txt" \
 && bash "$R/scripts/gpu_ab_cfgs.sh" "$TAG/ab" 2 bert-large "base:" "gm4:CLOUDTIK_AMD_GEMM_GROUP_M=4" "gm8:CLOUDTIK_AMD_GEMM_GROUP_M=8" \
      "blasdgrad:CLOUDTIK_AMD_ONETILE_GEMM="
rc=$?
[ $rc -eq 0 ] || { grep -E "FAIL|Error" "$O/tests.txt" | head; }
exit $rc
