#!/bin/bash
# r6: eight-wave interleaved GEMM (CLOUDTIK_AMD_GEMM_W4_DIAG=10: numerics + timing; 11: no DMA)
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r6t"; mkdir -p "$O"
cd "$R"
CLOUDTIK_AMD_GEMM_W4_DIAG=10 timeout -k 10 180 python -u bench/gemm_w4_probe.py > "$O/probe_10.jsonl" 2> "$O/probe_10.err"
rc=$?; cut -c1-300 "$O/probe_10.jsonl"; [ $rc -eq 0 ] || { tail -20 "$O/probe_10.err"; exit $rc; }
CLOUDTIK_AMD_GEMM_W4_DIAG=11 timeout -k 10 180 python -u bench/gemm_w4_probe.py --skip-check > "$O/probe_11.jsonl" 2> "$O/probe_11.err"
rc=$?; cat "$O/probe_11.jsonl"; [ $rc -eq 0 ] || { tail -20 "$O/probe_11.err"; exit $rc; }
