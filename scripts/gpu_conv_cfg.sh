#!/bin/bash
# conv configuration screen: GPU conv tests, then the per-shape probe over CFGS
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/convcfg"
mkdir -p "$O"
cd "$R"
timeout -k 10 300 python -u -m pytest tests/test_conv_igemm.py -m gpu -x -q --timeout 120 --timeout-method thread > "$O/tests.txt" 2>&1
rc=$?
tail -2 "$O/tests.txt"
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" "$O/tests.txt" | head -20; exit $rc; }
timeout -k 10 600 python -u bench/conv_igemm_probe.py --cfgs="${CFGS:--1,5,8,9,11,14,15}" > "$O/probe.md" 2> "$O/probe.err"
rc=$?
grep "cfg fwd" "$O/probe.err"
exit $rc
