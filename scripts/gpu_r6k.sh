#!/bin/bash
# r6: LayerNorm from-output backward -- kernel probe, LN GPU tests, step A/B.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r6k"; mkdir -p "$O"
cd "$R"
timeout -k 10 120 python -u bench/ln_from_y_probe.py > "$O/probe.json" 2> "$O/probe.err"
rc=$?; cat "$O/probe.json"; [ $rc -eq 0 ] || { tail -5 "$O/probe.err"; exit $rc; }
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_ops_gpu.py \
  tests/test_model_parity.py > "$O/tests.txt" 2>&1
rc=$?; tail -1 "$O/tests.txt"; [ $rc -eq 0 ] || exit $rc
bash "$R/scripts/gpu_ab_env.sh" r6k_ab CLOUDTIK_AMD_LN_FROM_Y "0 1" 2 bert-large
