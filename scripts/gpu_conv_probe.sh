#!/bin/bash
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/conv_probe"; mkdir -p "$OUT"
timeout -k 10 500 python3 "$R/bench/conv_igemm_probe.py" --cfgs="${CFGS:--1,0,1,4,5,6,7,8,9}" > "$OUT/probe.md" 2> "$OUT/probe.err" || { tail -20 "$OUT/probe.err"; exit 1; }
cat "$OUT/probe.md"
