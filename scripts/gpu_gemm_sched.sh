#!/bin/bash
# gemm_nt correctness + A/B of the DMA schedule variants (CLOUDTIK_AMD_GEMM_SCHED).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/${1:-gsched}"
mkdir -p "$OUT"
export PYTHONPATH="$R"
for s in ${SCHEDS:-0 1 2}; do
  CLOUDTIK_AMD_GEMM_SCHED=$s timeout -k 10 120 python -u -m pytest -x -q --timeout 60 --timeout-method thread "$R/tests/test_gemm_nt_gpu.py" > "$OUT/test_s$s.log" 2>&1 || { echo "sched $s tests failed"; tail -20 "$OUT/test_s$s.log"; exit 1; }
  echo "sched $s: $(tail -1 "$OUT/test_s$s.log")"
  CLOUDTIK_AMD_GEMM_SCHED=$s timeout -k 10 180 python -u "$R/bench/gemm_nt_probe.py" > "$OUT/probe_s$s.log" 2>&1 || { echo "sched $s probe failed"; tail -5 "$OUT/probe_s$s.log"; exit 1; }
  grep case "$OUT/probe_s$s.log" | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print('  ', d['case'], {k: v for k, v in d.items() if k.endswith('us') or k.endswith('tflops')})"
done
