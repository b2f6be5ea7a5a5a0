#!/bin/bash
# r5: new GEMM epilogue tests, BERT FFN derivative-storing epilogue A/B, gloo mixed-policy repeat.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=${1:-r5d}
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd "$R"
timeout -k 10 300 python -u -m pytest tests/test_gemm_nt_gpu.py tests/test_model_parity.py -m gpu -x -v --timeout 120 --timeout-method thread > "$O/gemm_tests.txt" 2>&1 \
 && tail -1 "$O/gemm_tests.txt" \
 && bash "$R/scripts/gpu_ab_env.sh" "$TAG/ab" CLOUDTIK_AMD_FFN_STORE_DGELU "0 1" 3 bert-large \
 && timeout -k 10 400 python -u bench.py --gpus 2 --dist-backend gloo --model all --steps 8 --warmup 2 --batch 64 --rn-batch 64 > "$O/gloo_mixed.log" 2> "$O/gloo_mixed.err" \
 && python - "$O/gloo_mixed.log" <<'PY'
import json, sys
d = json.loads([x for x in open(sys.argv[1]) if x.startswith("{")][-1])
print("gloo mixed: bert", d["step_ms"], "resnet", d["resnet50_step_ms"], d.get("resnet50_per_rank_step_ms"))
PY
rc=$?
[ $rc -eq 0 ] || { grep -E "FAIL|Error" "$O/gemm_tests.txt" | head; tail -20 "$O/gloo_mixed.err" 2>/dev/null; }
exit $rc
