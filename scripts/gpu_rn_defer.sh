#!/bin/bash
# ResNet tests + A/B of the deferred weight-gradient issue + a gap profile.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/rn_defer"; mkdir -p "$OUT"
cd "$R"
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_conv_igemm.py tests/test_model_parity.py -k "resnet or bottleneck or conv" > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
bash "$R/scripts/gpu_ab_cfgs.sh" rn_defer/ab 2 resnet50 "base:" "nodefer:CLOUDTIK_AMD_DEFER_WGRAD=0" || exit 1
for f in "$OUT"/ab/*.log; do echo "$(basename $f): $(grep -o '"resnet50_ms_per_step": [0-9.]*' $f)"; done
bash "$R/scripts/gpu_steady_rn.sh" rn_defer_gaps || exit 1
sed -n '/gap before/,/^$/p' "$R/gpurun_out/steady_rn/rn_defer_gaps.md" | head -12
