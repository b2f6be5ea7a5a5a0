#!/bin/bash
# r6: the tightened fp32 parity tests of the headline routing, then GEMM counter passes on the
# FFN1 shape (one-tile kernel vs hipBLASLt).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r6b"; mkdir -p "$O"
cd "$R"
timeout -k 10 300 python -u -m pytest tests/test_model_parity.py -m gpu -x -v --timeout 240 --timeout-method thread > "$O/parity.txt" 2>&1
rc=$?
tail -30 "$O/parity.txt" | grep -E "PASS|FAIL|Error|assert|passed|failed" | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash "$R/scripts/gpu_gemm_nt_pmc2.sh" r6b_pmc 32768 4096 1024 20
