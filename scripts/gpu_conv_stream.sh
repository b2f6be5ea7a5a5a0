#!/bin/bash
# Streamed persistent conv kernels (cfg 10-13): GPU tests, then the per-shape probe against the
# one-tile configurations and MIOpen with the roofline table.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/convstream"
mkdir -p "$O"
cd "$R"
timeout -k 10 300 python -u -m pytest tests/test_conv_igemm.py -m gpu -x -q --timeout 120 --timeout-method thread > "$O/tests.txt" 2>&1
rc=$?
tail -3 "$O/tests.txt"
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" "$O/tests.txt" | head -20; exit $rc; }
timeout -k 10 600 python -u bench/conv_igemm_probe.py --cfgs=-1,5,8,9,10,11,12,13 > "$O/probe.md" 2> "$O/probe.err"
rc=$?
tail -30 "$O/probe.md"
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 240 python -u bench.py --model resnet50 --steps 20 --warmup 5 > "$O/rn_$r.json" 2> "$O/rn_$r.err" || exit $?
  echo "resnet50 round $r: $(grep -o '"ms_per_step": [0-9.]*' "$O/rn_$r.json")"
done
