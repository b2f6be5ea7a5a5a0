#!/bin/bash
# r6: four-wave GEMM -- numerics + timing, then the no-DMA timing diagnostic.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r6m"; mkdir -p "$O"
cd "$R"
timeout -k 10 180 python -u bench/gemm_w4_probe.py > "$O/probe.jsonl" 2> "$O/probe.err"
rc=$?; cut -c1-400 "$O/probe.jsonl"; [ $rc -eq 0 ] || { tail -20 "$O/probe.err"; exit $rc; }
CLOUDTIK_AMD_GEMM_W4_DIAG=1 timeout -k 10 180 python -u bench/gemm_w4_probe.py --skip-check > "$O/probe_diag.jsonl" 2> "$O/probe_diag.err"
rc=$?; cat "$O/probe_diag.jsonl"; [ $rc -eq 0 ] || { tail -20 "$O/probe_diag.err"; exit $rc; }
