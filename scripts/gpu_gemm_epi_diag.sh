#!/bin/bash
# MFMA GEMM K-loop vs full kernel: probes with and without the epilogue's memory traffic
# (CLOUDTIK_AMD_GEMM_DIAG=4 skips the epilogue stores; results are wrong by design there)
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/gemm_epi"; mkdir -p "$OUT"
cd "$R"
for d in 0 4; do
  CLOUDTIK_AMD_GEMM_DIAG=$d PYTHONPATH=. timeout -k 10 240 python3 bench/gemm_nt_probe.py > "$OUT/nt_diag$d.jsonl" 2>&1 || { tail -5 "$OUT/nt_diag$d.jsonl"; exit 1; }
  CLOUDTIK_AMD_GEMM_DIAG=$d PYTHONPATH=. timeout -k 10 240 python3 bench/gemm_tn2_probe.py > "$OUT/tn2_diag$d.jsonl" 2>&1 || { tail -5 "$OUT/tn2_diag$d.jsonl"; exit 1; }
done
tail -n 3 "$OUT"/*.jsonl
