#!/bin/bash
# r6: paired-tile GEMM prototype -- numerics, then timing against the one-tile kernel and hipBLASLt.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r6e"; mkdir -p "$O"
cd "$R"
timeout -k 10 240 python -u bench/gemm_pp_probe.py --rounds 5 --iters 10 > "$O/probe.jsonl" 2> "$O/probe.err"
rc=$?
cat "$O/probe.jsonl" | cut -c1-1500
[ $rc -eq 0 ] || { tail -20 "$O/probe.err"; exit $rc; }
