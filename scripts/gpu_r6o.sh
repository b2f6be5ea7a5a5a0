#!/bin/bash
# r6: four-wave GEMM GPU tests + final timing of the kept (LDS-DMA) variant and its diagnostics.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r6o"; mkdir -p "$O"
cd "$R"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_w4_gpu.py > "$O/tests.txt" 2>&1
rc=$?; tail -2 "$O/tests.txt"; [ $rc -eq 0 ] || exit $rc
for d in 0 1 2; do
  CLOUDTIK_AMD_GEMM_W4_DIAG=$d timeout -k 10 180 python -u bench/gemm_w4_probe.py --skip-check > "$O/probe_$d.jsonl" 2> "$O/probe_$d.err"
  rc=$?; cat "$O/probe_$d.jsonl"; [ $rc -eq 0 ] || { tail -20 "$O/probe_$d.err"; exit $rc; }
done
