#!/bin/bash
# r6: four-wave GEMM variants: B-direct (diag 4, numerics + timing) and LDS-DMA (diag 0).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r6n"; mkdir -p "$O"
cd "$R"
for d in 4 0; do
  CLOUDTIK_AMD_GEMM_W4_DIAG=$d timeout -k 10 180 python -u bench/gemm_w4_probe.py > "$O/probe_$d.jsonl" 2> "$O/probe_$d.err"
  rc=$?; cut -c1-300 "$O/probe_$d.jsonl"; [ $rc -eq 0 ] || { tail -20 "$O/probe_$d.err"; exit $rc; }
done
