#!/bin/bash
# r6: after the DMA wait-state pad in the streamed conv kernel and the gemm_pp bias pin: conv and
# gemm_pp GPU tests, then three ResNet-50 bench runs.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r6s"; mkdir -p "$O"
cd "$R"
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_conv_igemm.py \
  tests/test_gemm_pp_gpu.py tests/test_resnet_train_entry.py > "$O/tests.txt" 2>&1
rc=$?; tail -1 "$O/tests.txt"; [ $rc -eq 0 ] || { grep -E "FAIL|Error" "$O/tests.txt" | head; exit $rc; }
for r in 1 2 3; do
  timeout -k 10 240 python -u bench.py --model resnet50 --steps 20 --warmup 5 --baseline-steps 0 > "$O/rn_$r.log" 2>&1 || exit 1
  python3 -c "
import json,sys
d=[json.loads(l) for l in open('$O/rn_$r.log') if l.startswith('{')][-1]
print('round $r', d['ms_per_step'], d['gpu_telemetry']['during']['sclk_mhz']['mean'])"
done
