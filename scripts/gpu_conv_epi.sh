#!/bin/bash
# Conv epilogue work: GPU conv tests, the epilogue cost probe, then ResNet-50 bench twice.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/convepi"
mkdir -p "$O"
cd "$R"
timeout -k 10 300 python -u -m pytest tests/test_conv_igemm.py tests/test_conv1x1.py tests/test_ops_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > "$O/tests.txt" 2>&1
rc=$?
tail -3 "$O/tests.txt"
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" "$O/tests.txt" | head -20; exit $rc; }
timeout -k 10 400 python -u bench/conv_epi_probe.py > "$O/probe.md" 2> "$O/probe.err" || { tail -5 "$O/probe.err"; exit 1; }
cat "$O/probe.md"
for r in 1 2; do
  timeout -k 10 240 python -u bench.py --model resnet50 --steps 20 --warmup 5 > "$O/rn_$r.json" 2> "$O/rn_$r.err" || exit $?
  echo "resnet50 round $r: $(grep -o '"ms_per_step": [0-9.]*' "$O/rn_$r.json")"
done
